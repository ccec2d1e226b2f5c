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
// extractor (ComputePyramid, Frame.cc:807-813).  The extractor leaves the device copy
// in a process-wide pool, indexed by the host level-0 buffer it was computed from; a
// later call that receives a Frame's host pyramid finds the device copy by that
// pointer.  The pool holds every host buffer it indexes (a copy of its cv::Mat
// header, i.e. a reference count), so an indexed buffer is never freed and handed to
// another image: a pointer hit is exact.  A buffer seen for the first time (a Frame
// deep-copied elsewhere, Frame.cc:186-188) is matched by one full compare of level 0,
// or uploaded.
#ifndef YGZFE_DROPIN_H_
#define YGZFE_DROPIN_H_

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <iterator>
#include <list>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <utility>
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

    // ORBextractor::ComputePyramid: the device pyramid of `img` (level 0, w x h, row
    // stride) computed by `ex` into a free entry.  The entry is found by pointer only
    // after bind() names the host level-0 buffer holding these pixels; until then it
    // can be found by content (its fingerprint, then a full compare).  The returned
    // frame stays valid until soft_capacity() newer pyramids have been made (unless pinned).
    ygzfe_frame *compute(ygzfe_extractor *ex, int nlevels, const uint8_t *img, int w, int h, size_t stride) {
        std::lock_guard<std::mutex> lk(mu_);
        Entry *e = slot(ex, nlevels, w, h);
        if (!e || !e->f) return failed(last_error());
        if (ygzfe_compute_pyramid(ex, e->f, img, (int)stride) != YGZFE_OK) return failed(last_error());
        set_fp(e, fingerprint(img, w, h, stride));
        return e->f;
    }

    // `level0` (a cv::Mat) holds the pixels `f`'s pyramid was computed from, and nothing
    // writes into it afterwards: held and indexed by its pointer
    template <class Mat>
    void bind(const ygzfe_frame *f, const Mat &level0) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = by_frame_.find(f);
        if (it != by_frame_.end() && level0.data) hold(it->second, level0);
    }

    // `dst` is a deep copy of `src` (Frame.cc:186-188, gpu::CopyImagePyramid): when
    // src's level 0 is indexed, dst's is indexed to the same device pyramid
    template <class MatVec>
    void alias(const MatVec &dst, const MatVec &src) {
        if (dst.empty() || src.empty() || !dst[0].data || !src[0].data) return;
        std::lock_guard<std::mutex> lk(mu_);
        auto ip = by_ptr_.find(src[0].data);
        if (ip == by_ptr_.end()) return;
        Entry *e = ip->second;
        if (dst[0].cols == e->w && dst[0].rows == e->h && (int)dst.size() == e->nlevels) hold(e, dst[0]);
    }

    // The device copy of a host pyramid (levels[l]: .data / .cols / .rows / .step).
    // An indexed level-0 pointer whose fingerprint still agrees is a hit; a buffer
    // seen for the first time is matched to an entry with the same fingerprint by one
    // full compare of level 0 against that entry's held pixels, else uploaded (one DMA).
    template <class MatVec>
    ygzfe_frame *find_or_upload(const MatVec &levels) {
        if (levels.empty() || !levels[0].data) {
            std::lock_guard<std::mutex> lk(mu_);
            return failed("empty mvImagePyramid");
        }
        const int w = levels[0].cols, h = levels[0].rows, nl = (int)levels.size();
        const uint8_t *key = levels[0].data;
        const size_t stride = (size_t)levels[0].step[0];
        std::lock_guard<std::mutex> lk(mu_);
        const uint64_t fp = fingerprint(key, w, h, stride);
        auto ip = by_ptr_.find(key);
        if (ip != by_ptr_.end()) {
            // a held buffer cannot be freed, but cv::Mat::create / copyTo of the same size
            // rewrites it in place: the pointer hit stands only while the fingerprint agrees
            Entry *e = ip->second;
            if (e->w == w && e->h == h && e->nlevels == nl && (!e->has_fp || e->fp == fp)) return touch(e)->f;
            release(e, key);  // rewritten: no longer this entry's pixels
        }
        auto range = by_fp_.equal_range(fp);
        for (auto it = range.first; it != range.second; ++it) {
            Entry *e = it->second;
            if (e->w == w && e->h == h && e->nlevels == nl && same_level0(*e, key, stride)) {
                hold(e, levels[0]);
                return touch(e)->f;
            }
        }
        ygzfe_extractor *ex = nullptr;
        for (auto it = live_.rbegin(); it != live_.rend() && !ex; ++it)
            if (it->second == nl) ex = it->first;
        if (!ex) return failed("no live ORBextractor with this pyramid's level count defines the level geometry");
        Entry *e = slot(ex, nl, w, h);
        if (!e || !e->f) return failed(last_error());
        std::vector<const uint8_t *> src(nl);
        std::vector<int> ss(nl);
        for (int l = 0; l < nl; l++) {
            src[l] = levels[l].data;
            ss[l] = (int)levels[l].step[0];
        }
        if (ygzfe_frame_set_levels(e->f, 0, nl, src.data(), ss.data()) != YGZFE_OK) return failed(last_error());
        set_fp(e, fp);
        hold(e, levels[0]);
        return e->f;
    }

    // Entries a caller needs together (a SearchLocalPointsDirect phase's keyframes)
    // are pinned: they are never recycled, and the pool grows past its soft capacity
    // rather than fail when every entry is pinned; it shrinks back once they are unpinned.
    void pin(const ygzfe_frame *f, int delta) {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = by_frame_.find(f);
        if (it == by_frame_.end()) return;
        it->second->pins += delta;
        if (delta < 0 && it->second->pins == 0) trim();
    }

    // why the last lookup returned no pyramid
    std::string why() {
        std::lock_guard<std::mutex> lk(mu_);
        return why_;
    }

    // pyramids a caller may hold unpinned at once (a newer lookup can recycle an older entry)
    static int soft_capacity() { return kCapacity; }
    int size() {
        std::lock_guard<std::mutex> lk(mu_);
        return (int)lru_.size();
    }
    // the most entries the pool has had at once (pinned growth past the soft capacity)
    int peak() {
        std::lock_guard<std::mutex> lk(mu_);
        return peak_;
    }
    // host level-0 buffers the pool holds (tests: the pool's host memory stays bounded)
    int held() {
        std::lock_guard<std::mutex> lk(mu_);
        return (int)by_ptr_.size();
    }

    // the extractors whose level geometry uploads use: the latest live one with the
    // pyramid's level count (a destroyed extractor -- e.g. Tracking's mpIniORBextractor
    // after initialization -- hands over to the one constructed before it)
    void set_extractor(ygzfe_extractor *ex, int nlevels) {
        std::lock_guard<std::mutex> lk(mu_);
        live_.push_back(std::make_pair(ex, nlevels));
    }
    void forget_extractor(ygzfe_extractor *ex) {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto it = lru_.begin(); it != lru_.end();)
            if (it->ex == ex) {
                it = destroy(it);
            } else {
                ++it;
            }
        for (auto it = live_.begin(); it != live_.end();)
            it = it->first == ex ? live_.erase(it) : it + 1;
    }

private:
    // a local map's keyframes plus the frames in flight: 96 pyramids of 752 x 480 are
    // ~46 MB of HBM; pinned entries may take the pool past it
    static constexpr int kCapacity = 96;
    // host buffers held per entry (the extractor's level 0, which the Frame shares, and
    // the copies Tracking makes, mLastFrame = Frame(mCurrentFrame), Tracking.cc:718); an
    // older one is released and, if met again, matched by content
    static constexpr int kHeld = 3;
    struct Held {
        const uint8_t *ptr;
        std::shared_ptr<const void> mat;  // the cv::Mat header copy that keeps the buffer alive
    };
    struct Entry {
        ygzfe_extractor *ex = nullptr;
        ygzfe_frame *f = nullptr;
        int w = 0, h = 0, nlevels = 0, pins = 0;
        uint64_t fp = 0;
        bool has_fp = false;
        std::vector<Held> held;  // host level-0 buffers with these pixels, oldest first
        std::list<Entry>::iterator self;  // its own position in lru_ (list iterators are stable)
    };
    static uint64_t mix(uint64_t h, uint64_t v) {
        h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
        return h * 0xBF58476D1CE4E5B9ull;
    }
    // the content index for first-seen buffers (a hit is confirmed by a full compare):
    // 8 whole rows (first, last, 6 spread) + 512 bytes on a stride coprime to the width
    static uint64_t fingerprint(const uint8_t *p, int w, int h, size_t stride) {
        uint64_t f = mix((uint64_t)w, (uint64_t)h);
        if (w <= 0 || h <= 0) return f;
        for (int k = 0; k < 8; k++) {
            const int y = k == 0 ? 0 : (k == 7 ? h - 1 : (int)((long)k * h / 7));
            const uint8_t *r = p + (size_t)y * stride;
            uint64_t acc = 0;
            int x = 0;
            for (; x + 8 <= w; x += 8) {
                uint64_t v;
                std::memcpy(&v, r + x, 8);
                acc = mix(acc, v);
            }
            for (; x < w; x++) acc = mix(acc, r[x]);
            f = mix(f, acc);
        }
        const size_t n = (size_t)w * h, step = n / 512 + 1;
        size_t i = 7 % n;
        for (int k = 0; k < 512; k++, i = (i + step * 2 + 1) % n) f = mix(f, p[(i / w) * stride + i % w]);
        return f;
    }
    // level 0 at p equals the entry's pixels (any held buffer: they are all equal)
    bool same_level0(const Entry &e, const uint8_t *p, size_t stride) const {
        if (e.held.empty()) return false;
        const Held &hb = e.held.back();
        const size_t hs = held_stride_.at(hb.ptr);
        for (int y = 0; y < e.h; y++)
            if (std::memcmp(hb.ptr + (size_t)y * hs, p + (size_t)y * stride, (size_t)e.w) != 0) return false;
        return true;
    }
    Entry *touch(Entry *e) {
        lru_.splice(lru_.begin(), lru_, e->self);
        return e;
    }
    template <class Mat>
    void hold(Entry *e, const Mat &m) {
        const uint8_t *p = m.data;
        auto ip = by_ptr_.find(p);
        if (ip != by_ptr_.end()) {
            if (ip->second == e) return;
            release(ip->second, p);  // a buffer the pool holds has one content: it moved entries
        }
        if ((int)e->held.size() >= kHeld) release(e, e->held.front().ptr);
        std::shared_ptr<const void> keep(new Mat(m), [](const void *q) { delete static_cast<const Mat *>(q); });
        e->held.push_back(Held{p, keep});
        by_ptr_[p] = e;
        held_stride_[p] = (size_t)m.step[0];
    }
    void release(Entry *e, const uint8_t *p) {
        for (auto it = e->held.begin(); it != e->held.end(); ++it)
            if (it->ptr == p) {
                e->held.erase(it);
                break;
            }
        auto ip = by_ptr_.find(p);
        if (ip != by_ptr_.end() && ip->second == e) {
            by_ptr_.erase(ip);
            held_stride_.erase(p);
        }
    }
    void unindex(Entry *e) {
        while (!e->held.empty()) release(e, e->held.back().ptr);
        if (e->has_fp) {
            auto range = by_fp_.equal_range(e->fp);
            for (auto it = range.first; it != range.second; ++it)
                if (it->second == e) {
                    by_fp_.erase(it);
                    break;
                }
            e->has_fp = false;
        }
    }
    void set_fp(Entry *e, uint64_t fp) {
        e->fp = fp;
        e->has_fp = true;
        by_fp_.insert(std::make_pair(fp, e));
    }
    std::list<Entry>::iterator destroy(std::list<Entry>::iterator it) {
        unindex(&*it);
        by_frame_.erase(it->f);
        ygzfe_frame_destroy(it->f);
        return lru_.erase(it);
    }
    // pinned entries made the pool grow: the unpinned least recently used ones beyond
    // the soft capacity are freed (device pyramid and held host buffers)
    void trim() {
        for (auto it = lru_.end(); (int)lru_.size() > kCapacity && it != lru_.begin();) {
            --it;
            if (it->pins == 0) it = destroy(it);
        }
    }
    // a free (least recently used, unpinned) entry for a w x h pyramid of `ex`, at the front:
    // the least recently used one of the same geometry if there is one (its device
    // pyramid is reused; another geometry's costs a hipFree + hipMalloc), else the LRU
    Entry *slot(ygzfe_extractor *ex, int nlevels, int w, int h) {
        auto victim = lru_.end();
        if ((int)lru_.size() >= kCapacity) {
            for (auto it = lru_.end(); it != lru_.begin();) {
                --it;
                if (it->pins == 0 && it->f && it->ex == ex && it->w == w && it->h == h) {
                    victim = it;
                    break;
                }
            }
            for (auto it = lru_.end(); victim == lru_.end() && it != lru_.begin();) {
                --it;
                if (it->pins == 0) victim = it;
            }
        }
        if (victim != lru_.end()) {
            lru_.splice(lru_.begin(), lru_, victim);
        } else {
            lru_.emplace_front();
            peak_ = std::max(peak_, (int)lru_.size());
        }
        Entry &e = lru_.front();
        e.self = lru_.begin();
        unindex(&e);
        if (!e.f || e.ex != ex || e.w != w || e.h != h) {
            by_frame_.erase(e.f);
            ygzfe_frame_destroy(e.f);
            e.f = nullptr;
            if (ygzfe_frame_create(ex, w, h, &e.f) != YGZFE_OK) e.f = nullptr;
            if (e.f) by_frame_[e.f] = &e;
        }
        e.ex = ex;
        e.w = w;
        e.h = h;
        e.nlevels = nlevels;
        e.pins = 0;
        return &e;
    }
    ygzfe_frame *failed(const char *why) {
        why_ = why ? why : "";
        return nullptr;
    }
    std::mutex mu_;
    std::string why_;
    int peak_ = 0;
    std::list<Entry> lru_;
    std::unordered_map<const uint8_t *, Entry *> by_ptr_;  // held host level-0 buffers
    std::unordered_map<const uint8_t *, size_t> held_stride_;
    std::unordered_multimap<uint64_t, Entry *> by_fp_;
    std::unordered_map<const ygzfe_frame *, Entry *> by_frame_;  // pin() / bind() lookups
    std::vector<std::pair<ygzfe_extractor *, int>> live_;  // (extractor, nlevels), construction order
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
