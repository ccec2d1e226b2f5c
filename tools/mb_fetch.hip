// mb_fetch.hip — calibrates PMC FETCH_SIZE on gfx950 for the load widths the
// ygzfe kernels use: streams a 256 MiB buffer once with 4-B (dword) and 16-B
// (dwordx4) coalesced loads and with 4-B buffer loads, one kernel per form;
// run under `rocprofv3 --pmc FETCH_SIZE` and compare each kernel's FETCH_SIZE
// (KiB) with the 262,144 KiB it reads.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_dword(const uint32_t *__restrict__ p, size_t n, uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_dwordx4(const uint4 *__restrict__ p, size_t n, uint32_t *__restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_buffer_dword(const uint32_t *__restrict__ p, uint32_t n, uint32_t *__restrict__ out) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, (int)(n * 4u), 0x00020000);
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        acc ^= __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * i, 0, 0);
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t bytes = 256ull << 20;
    uint32_t *p, *out;
    if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(p, 1, bytes);
    // flush L2/MALL between forms: touch another 1 GiB
    uint32_t *junk;
    if (hipMalloc(&junk, 1ull << 30) != hipSuccess) return 1;
    for (int rep = 0; rep < 2; rep++) {
        (void)hipMemset(junk, rep, 1ull << 30);
        hipLaunchKernelGGL(k_dword, dim3(2048), dim3(256), 0, 0, p, bytes / 4, out);
        (void)hipMemset(junk, rep + 2, 1ull << 30);
        hipLaunchKernelGGL(k_dwordx4, dim3(2048), dim3(256), 0, 0, (const uint4 *)p, bytes / 16, out);
        (void)hipMemset(junk, rep + 4, 1ull << 30);
        hipLaunchKernelGGL(k_buffer_dword, dim3(2048), dim3(256), 0, 0, p, (uint32_t)(bytes / 4), out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("mb_fetch: %zu KiB per kernel\n", bytes >> 10);
    return 0;
}
