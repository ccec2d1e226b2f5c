// slots.hip — fixed-size per-frame result slots of the offline sequence mode
// (MH01..05 sharded over the GPUs of a node, results
// gathered to rank 0 over RCCL).  One launch packs a rank's frames straight
// from the batch's keypoint / descriptor rows and the SparseImgAlign records
// into the slot buffer the gather sends, so no host round trip sits between
// the last kernel of the step and the collective.
//
// Slot layout (include/ygzfe.h YGZFE_SLOT_*; little endian, 16-B multiple):
//   [0, 64)            int32 n_kps, int32 n_visible, f32 q[4], f32 t[3],
//                      f32 chi2, int32 global frame, int32 has_align, 4 x 0
//   [64, 64 + 28 cap)  keypoint rows (cv::KeyPoint layout), rows >= n_kps zero
//   [.., + 32 cap)     descriptor rows, rows >= n_kps zero
//   zero padding to the slot size
// The align record of frame f is the pair (f-1 -> f): TCR of the frame
// relative to its predecessor (Tracking.cc:2171-2179); none for the first
// frame of the sequence.
#include "kernels.hpp"

namespace ygzfe {

__global__ __launch_bounds__(256) void k_pack_slots(const ygzfe_kp *__restrict__ kps, const uint8_t *__restrict__ desc,
                                                    const int *__restrict__ counts, int kp_cap,
                                                    const ygzfe_align_result *__restrict__ align, int frame_begin,
                                                    int global_first, uint8_t *__restrict__ slots, size_t slot_pitch) {
    const int j = blockIdx.x, f = frame_begin + j;
    const int n = min(max(counts[f], 0), kp_cap);
    uint32_t *s = reinterpret_cast<uint32_t *>(slots + (size_t)j * slot_pitch);
    const int t = threadIdx.x;
    if (t < 16) {
        uint32_t v = 0u;
        const bool has = align != nullptr && f >= 1;
        const ygzfe_align_result *a = has ? align + (f - 1) : nullptr;
        switch (t) {
            case 0: v = (uint32_t)n; break;
            case 1: v = has ? (uint32_t)a->n_visible : 0u; break;
            case 2: case 3: case 4: case 5:
                v = has ? __float_as_uint(a->T_cur_ref.q[t - 2]) : (t == 5 ? __float_as_uint(1.f) : 0u);
                break;
            case 6: case 7: case 8: v = has ? __float_as_uint(a->T_cur_ref.t[t - 6]) : 0u; break;
            case 9: v = has ? __float_as_uint(a->chi2) : 0u; break;
            case 10: v = (uint32_t)(global_first + j); break;
            case 11: v = has ? 1u : 0u; break;
            default: break;
        }
        s[t] = v;
    }
    // keypoint rows: 7 dwords each
    const uint32_t *ks = reinterpret_cast<const uint32_t *>(kps + (size_t)f * kp_cap);
    uint32_t *kd = s + 16;
    const int kw = 7 * kp_cap, kn = 7 * n;
    for (int i = t; i < kw; i += 256) kd[i] = i < kn ? ks[i] : 0u;
    // descriptor rows: 8 dwords each (16-B aligned in the batch)
    const uint4 *dsrc = reinterpret_cast<const uint4 *>(desc + (size_t)f * kp_cap * 32);
    uint32_t *dd = kd + kw;
    const int dw = 2 * kp_cap, dn = 2 * n;
    for (int i = t; i < dw; i += 256) {
        const uint4 v = i < dn ? dsrc[i] : make_uint4(0u, 0u, 0u, 0u);
        dd[4 * i] = v.x;
        dd[4 * i + 1] = v.y;
        dd[4 * i + 2] = v.z;
        dd[4 * i + 3] = v.w;
    }
    const int used = 16 + 15 * kp_cap, total = (int)(slot_pitch / 4);
    for (int i = used + t; i < total; i += 256) s[i] = 0u;
}

hipError_t launch_pack_slots(const ygzfe_kp *kps, const uint8_t *desc, const int *counts, int kp_cap,
                             const ygzfe_align_result *align, int frame_begin, int n_frames, int global_first,
                             uint8_t *slots, size_t slot_pitch, hipStream_t st) {
    if (n_frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_slots, dim3(n_frames), dim3(256), 0, st, kps, desc, counts, kp_cap, align, frame_begin,
                       global_first, slots, slot_pitch);
    return hipGetLastError();
}

}  // namespace ygzfe
