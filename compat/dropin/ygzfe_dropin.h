// ygzfe_dropin.h — shared state of the reference-signature drop-in headers
// (compat/dropin/ORBextractor.h, SparseImageAlign.h, Align.h, ORBmatcherGPU.h).
//
// These headers replace the reference's own headers of the same names: the
// reference's Tracking.cc / Frame.cc / ORBmatcher.cc keep calling
//   (*mpORBextractorLeft)(this, mvKeys, mDescriptors, ORBextractor::DSO_KEYPOINT)   Frame.cc:337
//   mpAlign->run(&mLastFrame, &mCurrentFrame, TCR)                                  Tracking.cc:2171
//   ygz::Align2D(curr->mvImagePyramid[search_level], ...)                            ORBmatcher.cc:1599
// unchanged, and the work runs on the GPU through include/ygzfe.h.  C++11 (the
// reference's -std=c++11, CMakeLists.txt:18-21); the Frame / MapPoint /
// KeyFrame types are template parameters read through the reference's own
// member names, so this header needs none of their definitions.
//
// Device pyramids: Frame::ComputeImagePyramid computes the pyramid through the
// extractor (ComputePyramid, then clones mvImagePyramid, Frame.cc:807-813).
// The extractor leaves the device copy in a small process-wide pool keyed by
// the level-0 bytes; a later call that receives the Frame's (cloned) host
// pyramid finds it there after one memcmp of level 0, and uploads the host
// levels only when the pool has no copy (a Frame built some other way).
#ifndef YGZFE_DROPIN_H_
#define YGZFE_DROPIN_H_

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <list>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "ygzfe.h"

namespace ygz {
namespace dropin {

inline int device() {
    const char *e = std::getenv("YGZFE_DEVICE");
    return e ? std::atoi(e) : 0;
}

// The reference never throws: failures become empty results;
// the last message is kept for the caller's logging.
inline const char *last_error() { return ygzfe_last_error(); }

// A failed call keeps the reference's empty-result convention, but says why on
// stderr once per (call site, message): Tracking would otherwise go LOST silently.
inline void log_once(const char *where, const char *why) {
    static std::mutex mu;
    static std::set<std::string> seen;
    std::lock_guard<std::mutex> lk(mu);
    std::string key = std::string(where) + ": " + (why ? why : "");
    if (seen.size() > 256 || !seen.insert(key).second) return;
    std::fprintf(stderr, "[ygzfe] %s failed: %s (returning the reference's empty result)\n", where, why ? why : "");
}

class PyramidPool {
public:
    static PyramidPool &instance() {
        static PyramidPool *p = new PyramidPool();  // lives as long as the process
        return *p;
    }

    // The device pyramid of `img` (level 0, w x h, row stride) computed by `ex`;
    // the returned frame stays valid until kCapacity newer pyramids have been made.
    ygzfe_frame *compute(ygzfe_extractor *ex, int nlevels, const uint8_t *img, int w, int h, size_t stride) {
        std::lock_guard<std::mutex> lk(mu_);
        Entry &e = slot(ex, nlevels, w, h);
        if (!e.f) return nullptr;
        e.level0.resize((size_t)w * h);
        for (int y = 0; y < h; y++) std::memcpy(&e.level0[(size_t)y * w], img + (size_t)y * stride, (size_t)w);
        if (ygzfe_compute_pyramid(ex, e.f, e.level0.data(), w) != YGZFE_OK) {
            e.level0.clear();
            return nullptr;
        }
        return e.f;
    }

    // The device copy of a host pyramid (levels[l]: .data / .cols / .rows / .step).
    // An entry whose level 0 last came from the same host pointer is checked
    // first (a KeyFrame shares its Frame's pyramid, KeyFrame.cc:257-260, so a
    // keyframe is found on its first entry); every hit is confirmed by a full
    // compare of level 0, so a reused host buffer never returns a stale pyramid.
    template <class MatVec>
    ygzfe_frame *find_or_upload(const MatVec &levels) {
        if (levels.empty()) return nullptr;
        const int w = levels[0].cols, h = levels[0].rows;
        const uint8_t *key = levels[0].data;
        std::lock_guard<std::mutex> lk(mu_);
        for (int pass = 0; pass < 2; pass++)
            for (auto it = lru_.begin(); it != lru_.end(); ++it) {
                if ((pass == 0) != (it->host_ptr == key)) continue;
                if (it->w == w && it->h == h && it->nlevels == (int)levels.size() && same_level0(*it, levels[0])) {
                    it->host_ptr = key;
                    lru_.splice(lru_.begin(), lru_, it);
                    return lru_.front().f;
                }
            }
        if (!ex_) return nullptr;  // no extractor yet: nothing defines the level geometry
        Entry &e = slot(ex_, (int)levels.size(), w, h);
        if (!e.f) return nullptr;
        for (int l = 0; l < (int)levels.size(); l++)
            if (ygzfe_frame_set_level(e.f, l, levels[l].data, (int)levels[l].step[0]) != YGZFE_OK) return nullptr;
        e.level0.resize((size_t)w * h);
        for (int y = 0; y < h; y++)
            std::memcpy(&e.level0[(size_t)y * w], levels[0].data + (size_t)y * levels[0].step[0], (size_t)w);
        e.host_ptr = key;
        return e.f;
    }

    // pyramids a caller may hold at once (a newer lookup can recycle an older entry)
    static int capacity() { return kCapacity; }

    // the extractor whose level geometry uploads use (the latest one constructed)
    void set_extractor(ygzfe_extractor *ex, int nlevels) {
        std::lock_guard<std::mutex> lk(mu_);
        ex_ = ex;
        nlevels_ = nlevels;
    }
    void forget_extractor(ygzfe_extractor *ex) {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto it = lru_.begin(); it != lru_.end();)
            if (it->ex == ex) {
                ygzfe_frame_destroy(it->f);
                it = lru_.erase(it);
            } else {
                ++it;
            }
        if (ex_ == ex) ex_ = nullptr;
    }

private:
    // a local map's keyframes (SearchLocalPointsDirect: <= 5 per map point, the
    // local keyframe set is capped at 80, Tracking.cc UpdateLocalKeyFrames) plus the
    // frames in flight: 96 pyramids of 752 x 480 are ~46 MB of HBM
    static constexpr int kCapacity = 96;
    struct Entry {
        ygzfe_extractor *ex = nullptr;
        ygzfe_frame *f = nullptr;
        int w = 0, h = 0, nlevels = 0;
        const uint8_t *host_ptr = nullptr;  // the host level 0 this content was last seen at
        std::vector<uint8_t> level0;
    };
    template <class Mat>
    static bool same_level0(const Entry &e, const Mat &m) {
        if (e.level0.size() != (size_t)e.w * e.h) return false;
        for (int y = 0; y < e.h; y++)
            if (std::memcmp(&e.level0[(size_t)y * e.w], m.data + (size_t)y * m.step[0], (size_t)e.w) != 0) return false;
        return true;
    }
    // a free (least recently used) entry for a w x h pyramid of `ex`, moved to the front
    Entry &slot(ygzfe_extractor *ex, int nlevels, int w, int h) {
        if ((int)lru_.size() >= kCapacity) {
            lru_.splice(lru_.begin(), lru_, std::prev(lru_.end()));
        } else {
            lru_.emplace_front();
        }
        Entry &e = lru_.front();
        if (!e.f || e.ex != ex || e.w != w || e.h != h) {
            ygzfe_frame_destroy(e.f);
            e.f = nullptr;
            if (ygzfe_frame_create(ex, w, h, &e.f) != YGZFE_OK) e.f = nullptr;
        }
        e.ex = ex;
        e.w = w;
        e.h = h;
        e.nlevels = nlevels;
        e.host_ptr = nullptr;
        e.level0.clear();
        return e;
    }
    std::mutex mu_;
    std::list<Entry> lru_;
    ygzfe_extractor *ex_ = nullptr;
    int nlevels_ = 0;
};

// cv::KeyPoint has the 28-byte ygzfe_kp layout (pt.x, pt.y, size, angle, response, octave, class_id)
template <class KeyPoint>
inline const ygzfe_kp *as_kp(const KeyPoint *p) {
    static_assert(sizeof(KeyPoint) == sizeof(ygzfe_kp), "cv::KeyPoint must have the 28-byte layout");
    return reinterpret_cast<const ygzfe_kp *>(p);
}
template <class KeyPoint>
inline ygzfe_kp *as_kp(KeyPoint *p) {
    static_assert(sizeof(KeyPoint) == sizeof(ygzfe_kp), "cv::KeyPoint must have the 28-byte layout");
    return reinterpret_cast<ygzfe_kp *>(p);
}

// rows [0, n) of a CV_8U N x 32 descriptor matrix, contiguous
template <class Mat>
inline std::vector<uint8_t> desc_rows(const Mat &m, int n) {
    std::vector<uint8_t> out((size_t)32 * (n > 0 ? n : 0));
    for (int i = 0; i < n; i++) std::memcpy(&out[(size_t)32 * i], m.data + (size_t)i * m.step[0], 32);
    return out;
}

}  // namespace dropin
}  // namespace ygz

#endif
