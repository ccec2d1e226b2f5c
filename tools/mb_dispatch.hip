// Residency / dispatch-rate microbenchmark: 256-thread workgroups that spin
// for ~SPIN_US microseconds with a given dynamic LDS size; per-block start/end
// (s_memrealtime, 100 MHz) -> peak concurrently resident workgroups.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_spin(unsigned long long *st, int spin_ticks, int vgpr_burn) {
    extern __shared__ unsigned char lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float acc = threadIdx.x;
    while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < spin_ticks) {
        for (int i = 0; i < vgpr_burn; i++) acc = acc * 1.0001f + 0.5f;
    }
    if (threadIdx.x == 0) {
        lds[0] = (unsigned char)acc;
        st[2 * blockIdx.x] = t0;
        st[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() + lds[0] * 0;
    }
}

int main() {
    const int nb = 16384;
    unsigned long long *d;
    (void)hipMalloc(&d, sizeof(unsigned long long) * 2 * nb);
    std::vector<unsigned long long> h(2 * nb);
    for (int kb : {0, 8, 22, 40}) {
        for (int spin_us : {2, 10}) {
            const size_t lds = (size_t)kb * 1024;
            hipLaunchKernelGGL(k_spin, dim3(nb), dim3(256), lds, 0, d, spin_us * 100, 1);
            (void)hipDeviceSynchronize();
            hipLaunchKernelGGL(k_spin, dim3(nb), dim3(256), lds, 0, d, spin_us * 100, 1);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * nb, hipMemcpyDeviceToHost);
            unsigned long long t0 = ~0ull, t1 = 0;
            for (int i = 0; i < nb; i++) { t0 = std::min(t0, h[2 * i]); t1 = std::max(t1, h[2 * i + 1]); }
            // peak concurrency via sweep
            std::vector<std::pair<unsigned long long, int>> ev;
            for (int i = 0; i < nb; i++) { ev.push_back({h[2 * i], 1}); ev.push_back({h[2 * i + 1], -1}); }
            std::sort(ev.begin(), ev.end());
            int cur = 0, peak = 0;
            double avg = 0;
            unsigned long long last = ev[0].first;
            for (auto &e : ev) { avg += (double)cur * (e.first - last); last = e.first; cur += e.second; peak = std::max(peak, cur); }
            avg /= (double)(t1 - t0);
            printf("LDS %2d KB spin %2d us: span %7.1f us  peak resident %5d  mean resident %7.1f  blocks/us %6.1f\n", kb,
                   spin_us, (t1 - t0) / 100.0, peak, avg, nb / ((t1 - t0) / 100.0));
        }
    }
    return 0;
}
