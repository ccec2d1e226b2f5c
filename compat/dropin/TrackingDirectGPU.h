// TrackingDirectGPU.h — the direct local-map search of Tracking on the GPU, read
// through the reference's own Frame / KeyFrame / MapPoint members.
//
// Tracking.cc includes Tracking_direct_gpu.inc in place of the body of
//   void Tracking::SearchLocalPointsDirect()                          Tracking.cc:2258-2410
// and ORBmatcher.cc forwards
//   bool ORBmatcher::FindDirectProjection(KeyFrame*, Frame*, MapPoint*, Vector2f&, int&)   ORBmatcher.cc:1573-1602
// through ORBmatcher_gpu.inc.  The caller-side filters (isBad, Frame::isInFrustum,
// SelectNearestKeyframe, UpdateLocalMap, the cache set) stay the reference's own
// host code; every (map point, keyframe) FindDirectProjection + Align2D of a phase
// runs in one batched GPU call (include/ygzfe.h ygzfe_search_local_points_direct),
// including the cache phase's sequential 5-px coverage grid, and the results are
// applied back to the Frame in the reference's order.
#ifndef YGZFE_TRACKING_DIRECT_GPU_H_
#define YGZFE_TRACKING_DIRECT_GPU_H_

#include <chrono>
#include <map>
#include <memory>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "Common.h"
#include "ygzfe_dropin.h"

namespace ygz {
namespace gpu {

template <class SE3>
inline ygzfe_se3 to_se3(const SE3 &T) {
    ygzfe_se3 o;
    o.q[0] = T.unit_quaternion().x();
    o.q[1] = T.unit_quaternion().y();
    o.q[2] = T.unit_quaternion().z();
    o.q[3] = T.unit_quaternion().w();
    for (int k = 0; k < 3; k++) o.t[k] = T.translation()[k];
    return o;
}

// Where a SearchLocalPointsDirect's time goes (read by tests/dropin/dropin_calls --time):
// pyramid-pool lookups, and the C-ABI calls (H2D, kernels, D2H); the rest is the
// reference's host loops (filters, SelectNearestKeyframe, item set-up, results).
struct DirectStats {
    double pool_ms = 0, call_ms = 0;
    long calls = 0;
};
inline DirectStats &direct_stats() {
    static DirectStats s;
    return s;
}
inline double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// One phase of SearchLocalPointsDirect: the points in the reference's loop order
// with their candidate observations (SelectNearestKeyframe order, <= 5 keyframes).
class DirectBatch {
public:
    DirectBatch() = default;
    DirectBatch(const DirectBatch &) = delete;
    DirectBatch &operator=(const DirectBatch &) = delete;
    ~DirectBatch() { release(); }

    void clear() {
        release();
        item_ptr_.assign(1, 0);
        ref_index_.clear();
        kps_.clear();
        pt_ref_.clear();
        T_cr_.clear();
        px_proj_.clear();
        kf_id_.clear();
        refs_.clear();
        slot_.clear();
        slot_tcr_.clear();
        slot_pose_.clear();
        ok_ = true;
    }

    // FindDirectProjection's inputs per observation (ORBmatcher.cc:1577-1582, 1530-1532):
    // kp = ref->mvKeys[index], pt_ref = ref->GetPose() * mp->GetWorldPos(),
    // TCR = curr->mTcw * ref->GetPose().inverse(); px_curr starts at (mTrackProjX, mTrackProjY)
    template <class MapPointT, class KeyFrameT, class FrameT>
    void add_point(MapPointT *mp, const std::vector<std::pair<KeyFrameT *, size_t>> &obs_sorted, FrameT &cur) {
        px_proj_.push_back(mp->mTrackProjX);
        px_proj_.push_back(mp->mTrackProjY);
        const auto pw = mp->GetWorldPos();
        for (auto &o : obs_sorted) {
            KeyFrameT *ref = o.first;
            // the keyframe's pose and TCR once per phase (a snapshot, as one GetPose() call)
            const int slot = slot_of(ref, cur);
            const auto &pose_ref = slot_pose<KeyFrameT>(slot);
            const auto pt_ref = pose_ref * pw;
            ref_index_.push_back(slot);
            kps_.push_back(*dropin::as_kp(&ref->mvKeys[o.second]));
            for (int k = 0; k < 3; k++) pt_ref_.push_back(pt_ref[k]);
            T_cr_.push_back(slot_tcr_[slot]);
            kf_id_.push_back((long)ref->mnId);
        }
        item_ptr_.push_back((int32_t)ref_index_.size());
    }
    int n_points() const { return (int)item_ptr_.size() - 1; }

    // one GPU call; false (and no matches) on any failure, with the message logged once
    template <class FrameT>
    bool run(FrameT &cur, int n_cache, int grid_size, int cache_hit_th, float border) {
        const int n = n_points();
        px_out_.assign(2 * (size_t)n + 2, 0.f);
        matched_.assign((size_t)n + 1, -1);
        status_.assign((size_t)n + 1, YGZFE_DIRECT_FAILED);
        cache_success_ = 0;
        local_ran_ = 1;
        if (!ok_) return fail("a keyframe pyramid could not be placed on the device");
        auto t0 = std::chrono::steady_clock::now();
        ygzfe_frame *cf = dropin::PyramidPool::instance().find_or_upload(cur.mvImagePyramid);
        direct_stats().pool_ms += ms_since(t0);
        if (!cf) return fail("the current frame pyramid could not be placed on the device");
        const ygzfe_camera cam{FrameT::fx, FrameT::fy, FrameT::cx, FrameT::cy};
        t0 = std::chrono::steady_clock::now();
        const int rc = ygzfe_search_local_points_direct(
            refs_.data(), (int)refs_.size(), cf, &cam, n_cache, n - n_cache, item_ptr_.data(), ref_index_.data(),
            kps_.data(), pt_ref_.data(), T_cr_.data(), px_proj_.data(), border, grid_size, cache_hit_th,
            px_out_.data(), matched_.data(), status_.data(), &cache_success_, &local_ran_);
        direct_stats().call_ms += ms_since(t0);
        direct_stats().calls++;
        release();  // the call has read the keyframe pyramids
        if (rc != YGZFE_OK) return fail(ygzfe_last_error());
        return true;
    }

    int status(int i) const { return status_[i]; }
    float px(int i, int k) const { return px_out_[2 * i + k]; }
    long matched_kf_id(int i) const { return kf_id_[matched_[i]]; }
    int cache_success() const { return cache_success_; }
    bool local_ran() const { return local_ran_ != 0; }

private:
    template <class KeyFrameT>
    using Pose = typename std::decay<decltype(std::declval<KeyFrameT &>().GetPose())>::type;
    template <class KeyFrameT>
    const Pose<KeyFrameT> &slot_pose(int slot) const {
        return *static_cast<const Pose<KeyFrameT> *>(slot_pose_[slot].get());
    }
    template <class KeyFrameT, class FrameT>
    int slot_of(KeyFrameT *ref, FrameT &cur) {
        auto it = slot_.find((const void *)ref);
        if (it != slot_.end()) return it->second;
        {
            auto *pose = new Pose<KeyFrameT>(ref->GetPose());
            slot_tcr_.push_back(to_se3(cur.mTcw * pose->inverse()));  // TCR (ORBmatcher.cc:1577-1582)
            slot_pose_.emplace_back(pose, [](const void *q) { delete static_cast<const Pose<KeyFrameT> *>(q); });
        }
        // every keyframe of the call stays resident until the call: pinned in the pool,
        // which grows past its soft capacity for a large local map instead of failing
        const auto t0 = std::chrono::steady_clock::now();
        ygzfe_frame *f = dropin::PyramidPool::instance().find_or_upload(ref->mvImagePyramid);
        direct_stats().pool_ms += ms_since(t0);
        if (!f) {
            if (ok_) dropin::log_once("SearchLocalPointsDirect: keyframe pyramid", dropin::PyramidPool::instance().why().c_str());
            ok_ = false;
        } else {
            dropin::PyramidPool::instance().pin(f, 1);
            pinned_.push_back(f);
        }
        const int s = (int)refs_.size();
        refs_.push_back(f);
        slot_[(const void *)ref] = s;
        return s;
    }
    void release() {
        for (const ygzfe_frame *f : pinned_) dropin::PyramidPool::instance().pin(f, -1);
        pinned_.clear();
    }
    bool fail(const char *why) {
        dropin::log_once("SearchLocalPointsDirect", why);
        return false;
    }
    std::vector<int32_t> item_ptr_{0}, ref_index_, matched_, status_;
    std::vector<ygzfe_kp> kps_;
    std::vector<float> pt_ref_, px_proj_, px_out_;
    std::vector<ygzfe_se3> T_cr_;
    std::vector<long> kf_id_;
    std::vector<const ygzfe_frame *> refs_, pinned_;
    std::unordered_map<const void *, int> slot_;
    std::vector<ygzfe_se3> slot_tcr_;
    std::vector<std::shared_ptr<const void>> slot_pose_;  // the keyframe poses, type-erased
    int cache_success_ = 0, local_ran_ = 1;
    bool ok_ = true;
};

// ORBmatcher::FindDirectProjection(ref, curr, mp, px_curr, search_level)
// (ORBmatcher.cc:1573-1602) for one (map point, keyframe) pair
template <class KeyFrameT, class FrameT, class MapPointT, class Vec2>
bool FindDirectProjection(KeyFrameT *ref, FrameT *curr, MapPointT *mp, Vec2 &px_curr, int &search_level) {
    const int index = (int)mp->GetObservations()[ref];
    const auto pose_ref = ref->GetPose();
    const auto TCR = curr->mTcw * pose_ref.inverse();
    const auto pt = pose_ref * mp->GetWorldPos();
    ygzfe_frame *rf = dropin::PyramidPool::instance().find_or_upload(ref->mvImagePyramid);
    ygzfe_frame *cf = dropin::PyramidPool::instance().find_or_upload(curr->mvImagePyramid);
    if (!rf || !cf) {
        dropin::log_once("FindDirectProjection", "a pyramid could not be placed on the device");
        return false;
    }
    const ygzfe_camera cam{FrameT::fx, FrameT::fy, FrameT::cx, FrameT::cy};
    const ygzfe_frame *refs[1] = {rf};
    const int32_t ri = 0;
    const float pt_ref[3] = {pt[0], pt[1], pt[2]};
    const ygzfe_se3 T = to_se3(TCR);
    float px[2] = {px_curr[0], px_curr[1]};
    int32_t level = 0;
    uint8_t ok = 0;
    if (ygzfe_find_direct_projection_batch(refs, cf, &cam, 1, &ri, dropin::as_kp(&ref->mvKeys[index]), pt_ref, &T, px,
                                           &level, &ok) != YGZFE_OK) {
        dropin::log_once("FindDirectProjection", ygzfe_last_error());
        return false;
    }
    search_level = level;
    px_curr[0] = px[0];
    px_curr[1] = px[1];
    return ok != 0;
}

}  // namespace gpu
}  // namespace ygz

#endif
