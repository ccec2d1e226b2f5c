// Align.h — drop-in replacement of the reference's include/Align.h (Align.h:20-26)
// over the gfx950 Align2D kernel (include/ygzfe.h ygzfe_align2d_image).
//
//   bool success = ygz::Align2D(curr->mvImagePyramid[search_level], _patch_with_border,
//                               _patch, 10, px_scaled);              ORBmatcher.cc:1599
// compiles unchanged: the level is a host cv::Mat, only the window around the
// estimate is uploaded (the whole level if the iterations walk out of it), and
// px / the converged flag come back as Align.cc:8-105 leaves them.
#ifndef YGZ_ALIGN_H_
#define YGZ_ALIGN_H_

#include "Common.h"
#include "ygzfe_dropin.h"

namespace ygz {

template <class Vec2>
bool Align2D(const cv::Mat &cur_img, uint8_t *ref_patch_with_border, uint8_t *ref_patch, const int n_iter,
             Vec2 &cur_px_estimate, bool no_simd = false) {
    (void)no_simd;
    float px[2] = {cur_px_estimate[0], cur_px_estimate[1]};
    uint8_t converged = 0;
    if (ygzfe_align2d_image(dropin::device(), cur_img.data, cur_img.cols, cur_img.rows, (int)cur_img.step[0],
                            ref_patch_with_border, ref_patch, n_iter, px, &converged) != YGZFE_OK)
        return false;
    cur_px_estimate[0] = px[0];
    cur_px_estimate[1] = px[1];
    return converged != 0;
}

}  // namespace ygz

#endif
