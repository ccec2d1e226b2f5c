// Microbenchmark: latency of the serial GN step (LDLT + SE3 exp + SE3 mul) in one lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../orb-ygz-slam_amd/csrc/align.hip"

using namespace ygzfe;
__global__ void k_mb(float *out, long long *cyc, int mode) {
    float Hm[36], b[6], x[6];
    for (int i = 0; i < 36; i++) Hm[i] = (i % 7 == 0) ? 100.f + i : 0.1f * (i % 5);
    for (int i = 0; i < 6; i++) b[i] = 0.01f * (i + 1);
    SE3 T;
    T.q[0] = T.q[1] = T.q[2] = 0; T.q[3] = 1; T.t[0] = T.t[1] = T.t[2] = 0;
    long long t0 = clock64();
    for (int it = 0; it < 30; it++) {
        if (mode & 1) ldlt_solve6_reg(Hm, b, x); else for (int k = 0; k < 6; k++) x[k] = b[k] * 0.001f;
        if (mode & 2) {
            float mx[6];
            for (int k = 0; k < 6; k++) mx[k] = -x[k];
            SE3 E, Tn;
            se3_exp(mx, E);
            se3_mul(T, E, Tn);
            T = Tn;
        }
        b[it % 6] += T.t[0] + x[0];
    }
    long long t1 = clock64();
    out[0] = T.q[0] + T.t[0] + x[0];
    cyc[0] = t1 - t0;
}
int main() {
    float *o; long long *c; hipMalloc(&o, 16); hipMalloc(&c, 16);
    for (int mode = 0; mode < 4; mode++) {
        k_mb<<<1, 64>>>(o, c, mode); hipDeviceSynchronize();
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipEventRecord(a); k_mb<<<1, 64>>>(o, c, mode); hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); long long cy; hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
        printf("mode %d (ldlt=%d exp=%d): %lld cycles for 30 steps (%.1f per step), kernel %.3f us\n", mode, mode & 1, (mode >> 1) & 1, cy, cy / 30.0, ms * 1e3);
    }
    return 0;
}
