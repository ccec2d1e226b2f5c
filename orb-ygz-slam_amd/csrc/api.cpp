// api.cpp — the C ABI of include/ygzfe.h over the gfx950 kernels.
//
// Host-side responsibilities only: planning (plan.cpp), device buffers,
// stream ordering and H2D/D2H of the host-pointer entry points.  No compute
// happens on the host; there is no CPU fallback.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kernels.hpp"
#include "plan.hpp"

namespace ygzfe {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

static const int kPatternHost[1024] = {
#include "../../include/ygzfe_pattern.inc"
};

static int ensure_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_error("no HIP device available (the ygzfe product path has no CPU fallback)");
        return YGZFE_EHIP;
    }
    if (device < 0 || device >= n) {
        set_error("device %d out of range (%d devices)", device, n);
        return YGZFE_EINVAL;
    }
    YGZ_HIP(hipSetDevice(device));
    static std::mutex mu;
    static bool uploaded[64] = {false};
    std::lock_guard<std::mutex> lk(mu);
    if (device < 64 && !uploaded[device]) {
        YGZ_HIP(upload_pattern(kPatternHost));
        uint32_t fails[2] = {0, 0};
        YGZ_HIP(run_arith_guard(fails));
        if (fails[0] || fails[1]) {
            set_error("arithmetic guard failed on device %d (f16 ordering: %u, cvRound: %u mismatches): the "
                      "library was built with flags that break its bit-exact paths (fast-math, denormal flush)",
                      device, fails[0], fails[1]);
            return YGZFE_EHIP;
        }
        uploaded[device] = true;
    }
    return YGZFE_OK;
}

// Graph capture vs. teardown across threads: a thread capturing its extraction
// graph must not overlap another thread's hipFree / stream / graph destruction (the
// runtime's capture bookkeeping is process-wide; tests/test_gpu_concurrency.py hit it
// with two extractors on two threads, Frame.cc:728-731).  Capture takes ~0.1 ms once
// per frame handle; teardown is rare: one lock for both.
static std::recursive_mutex &graph_mutex() {
    static std::recursive_mutex mu;
    return mu;
}

struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    bool owned = true;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p && owned) {
            std::lock_guard<std::recursive_mutex> lk(graph_mutex());  // not during another thread's capture
            (void)hipFree(p);
        }
        p = nullptr;
        n = 0;
        owned = true;
    }
    int ensure(size_t bytes) {
        if (owned && p && n >= bytes) return YGZFE_OK;
        if (!owned && p && n >= bytes) return YGZFE_OK;
        release();
        if (bytes == 0) bytes = 16;
        std::lock_guard<std::recursive_mutex> lk(graph_mutex());
        if (hipMalloc(&p, bytes) != hipSuccess) {
            p = nullptr;
            set_error("hipMalloc(%zu) failed", bytes);
            return YGZFE_ENOMEM;
        }
        n = bytes;
        // YGZFE_POISON=1 (debugging): fresh buffers start as 0xA5 bytes instead of whatever
        // the allocator hands back, so a read-before-write shows on every run
        static const bool poison = getenv("YGZFE_POISON") != nullptr;
        if (poison) (void)hipMemset(p, 0xA5, bytes);
        return YGZFE_OK;
    }
    void bind(void *ext, size_t bytes) {
        release();
        p = ext;
        n = bytes;
        owned = false;
    }
    template <class T>
    T *as() const { return reinterpret_cast<T *>(p); }
};

// page-locked host staging (hipHostMalloc): one DMA per direction per call
// instead of a pageable copy per argument
struct HostBuf {
    void *p = nullptr;
    size_t n = 0;
    HostBuf() = default;
    HostBuf(const HostBuf &) = delete;
    HostBuf &operator=(const HostBuf &) = delete;
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
    int ensure(size_t bytes) {
        if (p && n >= bytes) return YGZFE_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        bytes = std::max<size_t>(bytes, 4096);
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            set_error("hipHostMalloc(%zu) failed", bytes);
            return YGZFE_ENOMEM;
        }
        n = bytes;
        return YGZFE_OK;
    }
    template <class T>
    T *as() const { return reinterpret_cast<T *>(p); }
};

static inline size_t align16(size_t v) { return (v + 15) & ~(size_t)15; }

// Host entry points without a handle (Hamming, RGB-D depth lookup, Align2D on a host
// image, FAST-10 ROIs): a call leases a staging area from a process-wide pool per
// device -- its own non-blocking stream, a device buffer and pinned in / out buffers
// that only grow -- and returns it when the call ends, so a call is one packed H2D,
// the launches, one packed D2H and one stream synchronisation (no allocation, no
// device-wide synchronisation).  The pool holds as many areas as calls ever ran at
// once, whatever the number of threads that come and go (no per-thread leak).
struct CallStaging {
    hipStream_t stream = nullptr;
    DevBuf dev;
    HostBuf hin, hout;
};
static std::mutex &staging_mutex() {
    static std::mutex mu;
    return mu;
}
static std::map<int, std::vector<CallStaging *>> &staging_free() {
    static auto *pool = new std::map<int, std::vector<CallStaging *>>();  // lives with the process
    return *pool;
}
struct StagingLease {
    CallStaging *s = nullptr;
    int device = -1;
    StagingLease() = default;
    StagingLease(const StagingLease &) = delete;
    StagingLease &operator=(const StagingLease &) = delete;
    ~StagingLease() {
        if (!s) return;
        // an early error return may leave DMAs into / out of the pinned buffers queued:
        // the next lessee (possibly another thread) writes them at once
        if (hipStreamQuery(s->stream) != hipSuccess) (void)hipStreamSynchronize(s->stream);
        std::lock_guard<std::mutex> lk(staging_mutex());
        staging_free()[device].push_back(s);
    }
    CallStaging *operator->() const { return s; }
    int acquire(int dev) {
        device = dev;
        {
            std::lock_guard<std::mutex> lk(staging_mutex());
            std::vector<CallStaging *> &fl = staging_free()[dev];
            if (!fl.empty()) {
                s = fl.back();
                fl.pop_back();
                return YGZFE_OK;
            }
        }
        CallStaging *n = new CallStaging();
        if (hipStreamCreateWithFlags(&n->stream, hipStreamNonBlocking) != hipSuccess) {
            delete n;
            set_error("hipStreamCreate failed");
            return YGZFE_EHIP;
        }
        s = n;
        return YGZFE_OK;
    }
};

#define YGZ_TRY(x)                          \
    do {                                    \
        int r_ = (x);                       \
        if (r_ != YGZFE_OK) return r_;      \
    } while (0)

struct PlanDev {
    PlanHost host;
    DevBuf plan, cells, tabs;
    int upload() {
        YGZ_TRY(plan.ensure(sizeof(Plan)));
        YGZ_TRY(cells.ensure(sizeof(CellDesc) * (host.cells.size() + 1)));
        YGZ_TRY(tabs.ensure(sizeof(int) * host.tabs.size()));
        host.plan.dtabs = tabs.as<int32_t>();
        YGZ_HIP(hipMemcpy(plan.p, &host.plan, sizeof(Plan), hipMemcpyHostToDevice));
        if (!host.cells.empty())
            YGZ_HIP(hipMemcpy(cells.p, host.cells.data(), sizeof(CellDesc) * host.cells.size(), hipMemcpyHostToDevice));
        YGZ_HIP(hipMemcpy(tabs.p, host.tabs.data(), sizeof(int) * host.tabs.size(), hipMemcpyHostToDevice));
        return YGZFE_OK;
    }
    const Plan &hp() const { return host.plan; }
    const Plan *dp() const { return plan.as<Plan>(); }
};

static int make_plan(const ygzfe_orb_params &p, int W, int H, std::unique_ptr<PlanDev> *out) {
    std::unique_ptr<PlanDev> pd(new PlanDev());
    char err[256];
    if (build_plan(p, W, H, &pd->host, err, sizeof(err)) != 0) {
        set_error("%s", err);
        return YGZFE_EINVAL;
    }
    YGZ_TRY(pd->upload());
    *out = std::move(pd);
    return YGZFE_OK;
}

// extraction scratch for F frames of one plan
struct Workspace {
    int F = 0, rows = 0;
    DevBuf blur, cellbuf, cellcnt, candA, candB, sel, selcnt, kps, desc, counts, nexist, err, ojobs, octq;
    DevBuf occ, dso_keys, dso_cnt, dso_total;
    int ensure(const Plan &P, int frames, int rows_needed) {
        F = frames;
        rows = rows_needed;
        YGZ_TRY(blur.ensure((size_t)F * P.pyr_bytes));
        YGZ_TRY(cellbuf.ensure((size_t)F * P.ncells * P.cell_cap * 4 + 16));
        YGZ_TRY(cellcnt.ensure((size_t)F * P.ncells * 4 + 16));
        YGZ_TRY(candA.ensure((size_t)F * P.cand_total * 8 + 16));
        YGZ_TRY(candB.ensure((size_t)F * P.cand_total * 8 + 16));
        YGZ_TRY(sel.ensure((size_t)F * P.sel_total * 4 + 16));
        YGZ_TRY(ojobs.ensure((size_t)F * P.sel_total * 8 + 16));
        YGZ_TRY(selcnt.ensure((size_t)F * P.nlevels * 4 + 128));  // tail: k_orient_desc's 8-int scalar load
        YGZ_TRY(kps.ensure((size_t)F * rows * sizeof(ygzfe_kp) + 16));
        YGZ_TRY(desc.ensure((size_t)F * rows * 32 + 16));
        YGZ_TRY(counts.ensure((size_t)F * 4 + 16));
        YGZ_TRY(nexist.ensure((size_t)F * 4 + 16));
        YGZ_TRY(err.ensure(16));
        YGZ_TRY(octq.ensure(octree_queue_ints(P, F) * sizeof(int)));
        return YGZFE_OK;
    }
};

}  // namespace ygzfe

using namespace ygzfe;

// --------------------------------------------------------------------------- handles
struct ygzfe_extractor {
    ygzfe_orb_params p;
    int device = 0;
    // frames borrow the extractor (its stream, mutex, plans): a destroy while frames are
    // alive is deferred to the last frame's destroy (under graph_mutex())
    int live_frames = 0;
    bool dead = false;
    hipStream_t stream = nullptr;
    ScaleInfo scales;
    std::map<std::pair<int, int>, std::unique_ptr<PlanDev>> plans;
    Workspace ws;
    int dso_grid = -1;
    // SearchLocalPointsDirect staging: one packed H2D, one packed D2H per call
    DevBuf direct_dev;
    HostBuf direct_hin, direct_hout;
    // single-frame latency path: side streams (side[0] the blur, side[1] the octree
    // classes after the first under YGZFE_OCT_FORK) forked from / joined to `stream`, pinned staging,
    // the packed extraction result (one D2H) and the SparseImgAlign buffers
    hipStream_t side[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_join[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_oct_fork = nullptr, ev_oct_join[2] = {nullptr, nullptr};
    HostBuf hin, hout, himg;
    hipEvent_t ev_img = nullptr;  // the last image DMA out of himg
    DevBuf res, align_in, align_scratch, align_out;
    // SparseImgAlign in flight (ygzfe_sparse_align_begin / _end): its own stream,
    // pinned staging and completion event, so it overlaps the same frame's extraction
    hipStream_t astream = nullptr;
    hipEvent_t ev_align_fork = nullptr, ev_align_done = nullptr;
    HostBuf ahin, ahout;
    HostBuf hlvl;  // page-locked staging of ygzfe_frame_level / _set_level (pageable 2-D copies are row by row)
    bool align_pending = false;
    bool graph_broken = false;  // stream capture failed once: plain launches
    std::mutex mu;
    // -1 when neither `stream` nor a side stream is in a capture, else the first that is
    // (0: stream, 1..3: side[0..2])
    int capture_left_open() const {
        const hipStream_t all[4] = {stream, side[0], side[1], side[2]};
        for (int i = 0; i < 4; i++) {
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            if (all[i] && (hipStreamIsCapturing(all[i], &cs) != hipSuccess || cs != hipStreamCaptureStatusNone))
                return i;
        }
        return -1;
    }
    int ensure_side() {
        if (side[0]) return YGZFE_OK;
        for (int i = 0; i < 3; i++) {
            YGZ_HIP(hipStreamCreateWithFlags(&side[i], hipStreamNonBlocking));
            YGZ_HIP(hipEventCreateWithFlags(&ev_join[i], hipEventDisableTiming));
        }
        YGZ_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
        YGZ_HIP(hipEventCreateWithFlags(&ev_oct_fork, hipEventDisableTiming));
        YGZ_HIP(hipEventCreateWithFlags(&ev_img, hipEventDisableTiming));
        for (int i = 0; i < 2; i++) YGZ_HIP(hipEventCreateWithFlags(&ev_oct_join[i], hipEventDisableTiming));
        return YGZFE_OK;
    }
    // Does work on `cand` run beside work on `stream`?  `stream` is held for 2 ms by
    // one lane; an empty kernel on `cand` must finish inside the hold.  A stream that
    // shares the hardware queue of `stream` waits for the hold instead.
    int probe_beside(hipStream_t cand, bool &beside) {
        beside = false;
        YGZ_HIP(launch_empty(cand));  // the candidate's queue acquired, both streams idle
        YGZ_HIP(hipStreamSynchronize(cand));
        YGZ_HIP(hipStreamSynchronize(stream));
        hipEvent_t ea = nullptr, eb = nullptr;
        hipError_t e = hipEventCreateWithFlags(&ea, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&eb, hipEventDisableTiming);
        if (e == hipSuccess) e = launch_hold_us(2000, stream);
        if (e == hipSuccess) e = hipEventRecord(ea, stream);
        if (e == hipSuccess) e = launch_empty(cand);
        if (e == hipSuccess) e = hipEventRecord(eb, cand);
        if (e == hipSuccess) {
            const auto t0 = std::chrono::steady_clock::now();
            while (hipEventQuery(eb) == hipErrorNotReady &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(50))
                std::this_thread::yield();
            beside = hipEventQuery(eb) == hipSuccess && hipEventQuery(ea) == hipErrorNotReady;
        }
        (void)hipStreamSynchronize(stream);
        (void)hipStreamSynchronize(cand);
        if (ea) (void)hipEventDestroy(ea);
        if (eb) (void)hipEventDestroy(eb);
        if (e != hipSuccess) { set_error("align stream probe: %s", hipGetErrorString(e)); return YGZFE_EHIP; }
        return YGZFE_OK;
    }
    int ensure_align_stream() {
        if (astream) return YGZFE_OK;
        // Normal priority, created on first use.  Measured alternatives (tools/run_lat_ab.sh):
        // the greatest / least priority, a dedicated queue (full CU mask) and creating the
        // extractor's streams eagerly all ran the single-frame path 15-30 % slower.
        // Streams beyond GPU_MAX_HW_QUEUES share hardware queues, and an align stream on the
        // extraction stream's queue runs after the extraction instead of beside it (0.28
        // instead of 0.16 ms per frame).  So each candidate is probed; a
        // rejected one stays alive until the choice is made (the next stream then lands on
        // another queue).  YGZFE_ALIGN_PROBE=0 keeps the first stream unprobed.
        YGZ_HIP(hipEventCreateWithFlags(&ev_align_fork, hipEventDisableTiming));
        YGZ_HIP(hipEventCreateWithFlags(&ev_align_done, hipEventDisableTiming));
        const char *pe = getenv("YGZFE_ALIGN_PROBE");
        const bool probe = !(pe && pe[0] == '0');
        std::vector<hipStream_t> rejected;
        int rc = YGZFE_OK;
        // at most 4 probes and 150 ms in all (another thread's work on the GPU can make
        // good candidates fail); then the next stream is taken unprobed
        const auto t_start = std::chrono::steady_clock::now();
        for (int attempt = 0; rc == YGZFE_OK && !astream; attempt++) {
            hipStream_t s = nullptr;
            if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
                set_error("hipStreamCreate failed");
                rc = YGZFE_EHIP;
                break;
            }
            bool beside = true;
            const bool in_budget = std::chrono::steady_clock::now() - t_start < std::chrono::milliseconds(150);
            const bool probed = probe && attempt < 4 && in_budget;
            if (probed) rc = probe_beside(s, beside);
            if (rc == YGZFE_OK && beside) {
                astream = s;
                align_probe_beside = probed ? 1 : 0;
            } else {
                rejected.push_back(s);
            }
            align_probe_attempts = attempt + 1;
        }
        for (hipStream_t s : rejected) (void)hipStreamDestroy(s);
        return rc;
    }
    int align_probe_attempts = 0;  // streams created by the placement probe (0: no align yet)
    int align_probe_beside = -1;   // 1: the align stream passed the probe; 0: taken unprobed
    // work about to rewrite a pyramid on `st` waits for the alignment reading it
    int order_after_align(hipStream_t st) {
        if (align_pending) YGZ_HIP(hipStreamWaitEvent(st, ev_align_done, 0));
        return YGZFE_OK;
    }
};

struct ygzfe_frame {
    ygzfe_extractor *ex = nullptr;
    PlanDev *plan = nullptr;
    int W = 0, H = 0;
    DevBuf pyr;
    // the captured single-frame extraction (ygzfe_extract, no existing rows)
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    const void *gkey[15] = {};
    int grows = 0;
    size_t gcopy = 0;
    void drop_graph() {
        if (gexec) (void)hipGraphExecDestroy(gexec);
        if (graph) (void)hipGraphDestroy(graph);
        gexec = nullptr;
        graph = nullptr;
    }
    ~ygzfe_frame() { drop_graph(); }
};

struct ygzfe_batch {
    ygzfe_orb_params p;
    int device = 0;
    int maxF = 0;
    hipStream_t stream = nullptr;
    // fork/join inside one extract: the FAST levels >= 1 overlap level 0
    hipStream_t aux[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_join[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_oct_fork = nullptr, ev_oct_join[2] = {nullptr, nullptr};
    // end of the last extraction's descriptor pass (the last reader of the pyramid,
    // FAST / octree scratch): the next extraction and uploads wait on it
    hipEvent_t ev_desc_done = nullptr;
    bool desc_pending = false;
    std::unique_ptr<PlanDev> plan;
    DevBuf pyr;
    Workspace ws;
    // align scratch
    DevBuf jobs, ascratch, pairs_tmp;
    size_t ascratch_per_job = 0;
    // stereo scratch: jobs + winning SADs [pairs][kp_cap]
    DevBuf sjobs, ssad;
    // BoW scratch: per-feature word / weight / node [frames][kp_cap]
    DevBuf bow_word, bow_weight, bow_nid;
    // per-stage kernel timing with hipEvents on the launch stream (no sync while recording)
    bool timing = false;
    std::vector<hipEvent_t> pool;
    struct Rec { int stage; hipEvent_t a, b; };
    std::vector<Rec> pending;
    double total_ms[16] = {0};
    long calls[16] = {0};
    hipEvent_t get_event() {
        hipEvent_t e = nullptr;
        if (!pool.empty()) { e = pool.back(); pool.pop_back(); }
        else if (hipEventCreate(&e) != hipSuccess) e = nullptr;
        return e;
    }
    hipEvent_t begin(hipStream_t st) {
        if (!timing) return nullptr;
        hipEvent_t a = get_event();
        if (a) (void)hipEventRecord(a, st);
        return a;
    }
    void end(int stage, hipEvent_t a, hipStream_t st) {
        if (!timing || !a) return;
        hipEvent_t e = get_event();
        if (!e) return;
        (void)hipEventRecord(e, st);
        pending.push_back({stage, a, e});
    }
    int collect() {
        for (auto &r : pending) {
            float ms = 0.f;
            YGZ_HIP(hipEventSynchronize(r.b));
            YGZ_HIP(hipEventElapsedTime(&ms, r.a, r.b));
            total_ms[r.stage] += ms;
            calls[r.stage] += 1;
            pool.push_back(r.a);
            pool.push_back(r.b);
        }
        pending.clear();
        return YGZFE_OK;
    }
};

static const char *kStageNames[] = {"pyramid", "blur7", "fast9_cells", "octree", "orient_rbrief", "hamming_best2",
                                    "sparse_align", "stereo", "pack_slots"};
constexpr int kNumStages = 9;
enum { ST_PYR, ST_BLUR, ST_FAST, ST_OCT, ST_DESC, ST_HAM, ST_ALIGN, ST_STEREO, ST_PACK };

extern "C" {

const char *ygzfe_last_error(void) { return g_err; }

int ygzfe_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ygzfe_descriptor_distance(const uint8_t *a, const uint8_t *b) {
    // ORBmatcher::DescriptorDistance (ORBmatcher.cc:1507-1523): host scalar helper.
    int d = 0;
    for (int i = 0; i < 32; i += 4) {
        uint32_t x, y;
        memcpy(&x, a + i, 4);
        memcpy(&y, b + i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

// ------------------------------------------------------------------ extractor
int ygzfe_extractor_create(const ygzfe_orb_params *p, int device, ygzfe_extractor **out) {
    if (!p || !out) { set_error("null argument"); return YGZFE_EINVAL; }
    if (p->nlevels < 1 || p->nlevels > YGZFE_MAX_LEVELS || !(p->scale_factor > 1.0f) || p->nfeatures < 0) {
        set_error("invalid ORB parameters");
        return YGZFE_EINVAL;
    }
    YGZ_TRY(ensure_device(device));
    std::unique_ptr<ygzfe_extractor> ex(new ygzfe_extractor());
    ex->p = *p;
    ex->device = device;
    orb_scales(*p, &ex->scales);
    YGZ_HIP(hipStreamCreateWithFlags(&ex->stream, hipStreamNonBlocking));
    *out = ex.release();
    return YGZFE_OK;
}

static void extractor_release(ygzfe_extractor *ex) {
    (void)hipSetDevice(ex->device);
    if (ex->stream) (void)hipStreamSynchronize(ex->stream);
    for (int i = 0; i < 3; i++) {
        if (ex->side[i]) (void)hipStreamSynchronize(ex->side[i]), (void)hipStreamDestroy(ex->side[i]);
        if (ex->ev_join[i]) (void)hipEventDestroy(ex->ev_join[i]);
    }
    if (ex->ev_fork) (void)hipEventDestroy(ex->ev_fork);
    if (ex->astream) {
        (void)hipStreamSynchronize(ex->astream);
        (void)hipStreamDestroy(ex->astream);
        (void)hipEventDestroy(ex->ev_align_fork);
        (void)hipEventDestroy(ex->ev_align_done);
    }
    if (ex->ev_img) (void)hipEventDestroy(ex->ev_img);
    if (ex->ev_oct_fork) (void)hipEventDestroy(ex->ev_oct_fork);
    for (int i = 0; i < 2; i++)
        if (ex->ev_oct_join[i]) (void)hipEventDestroy(ex->ev_oct_join[i]);
    ex->plans.clear();
    if (ex->stream) (void)hipStreamDestroy(ex->stream);
    delete ex;
}

void ygzfe_extractor_destroy(ygzfe_extractor *ex) {
    if (!ex) return;
    std::lock_guard<std::recursive_mutex> lk(graph_mutex());
    if (ex->live_frames > 0) {  // released by the last frame (a finalizer order we do not control)
        ex->dead = true;
        return;
    }
    extractor_release(ex);
}

int ygzfe_orb_plan(const ygzfe_orb_params *p, int width, int height, int32_t *level_w, int32_t *level_h,
                   int32_t *budget, int32_t *ncells, int32_t *umax) {
    if (!p) { set_error("null argument"); return YGZFE_EINVAL; }
    PlanHost ph;
    char err[256];
    if (build_plan(*p, width, height, &ph, err, sizeof(err)) != 0) { set_error("%s", err); return YGZFE_EINVAL; }
    for (int l = 0; l < ph.plan.nlevels; l++) {
        if (level_w) level_w[l] = ph.plan.lv[l].w;
        if (level_h) level_h[l] = ph.plan.lv[l].h;
        if (budget) budget[l] = ph.plan.lv[l].budget;
        if (ncells) ncells[l] = ph.plan.lv[l].ncells;
    }
    if (umax)
        for (int i = 0; i < 16; i++) umax[i] = ph.plan.umax[i];
    return YGZFE_OK;
}

int ygzfe_extractor_levels(const ygzfe_extractor *ex, int *nlevels, float *scale, float *inv_scale,
                           float *sigma2, float *inv_sigma2) {
    if (!ex) { set_error("null extractor"); return YGZFE_EINVAL; }
    const int L = ex->p.nlevels;
    if (nlevels) *nlevels = L;
    for (int i = 0; i < L; i++) {
        if (scale) scale[i] = ex->scales.scale[i];
        if (inv_scale) inv_scale[i] = ex->scales.inv_scale[i];
        if (sigma2) sigma2[i] = ex->scales.sigma2[i];
        if (inv_sigma2) inv_sigma2[i] = ex->scales.inv_sigma2[i];
    }
    return YGZFE_OK;
}

int ygzfe_extractor_features_per_level(const ygzfe_extractor *ex, int32_t *out) {
    if (!ex || !out) { set_error("null argument"); return YGZFE_EINVAL; }
    for (int i = 0; i < ex->p.nlevels; i++) out[i] = ex->scales.budget[i];
    return YGZFE_OK;
}

int ygzfe_extractor_dso_grid(ygzfe_extractor *ex, int32_t *get, const int32_t *set) {
    if (!ex) { set_error("null extractor"); return YGZFE_EINVAL; }
    if (get) *get = ex->dso_grid;
    if (set) ex->dso_grid = *set;
    return YGZFE_OK;
}

static int extractor_plan(ygzfe_extractor *ex, int W, int H, PlanDev **out) {
    auto key = std::make_pair(W, H);
    auto it = ex->plans.find(key);
    if (it == ex->plans.end()) {
        std::unique_ptr<PlanDev> pd;
        YGZ_TRY(make_plan(ex->p, W, H, &pd));
        it = ex->plans.emplace(key, std::move(pd)).first;
    }
    *out = it->second.get();
    return YGZFE_OK;
}

int ygzfe_frame_create(ygzfe_extractor *ex, int width, int height, ygzfe_frame **out) {
    if (!ex || !out) { set_error("null argument"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    std::unique_ptr<ygzfe_frame> f(new ygzfe_frame());
    f->ex = ex;
    f->W = width;
    f->H = height;
    YGZ_TRY(extractor_plan(ex, width, height, &f->plan));
    YGZ_TRY(f->pyr.ensure(f->plan->hp().pyr_bytes));
    {
        std::lock_guard<std::recursive_mutex> g(graph_mutex());
        ex->live_frames++;
    }
    *out = f.release();
    return YGZFE_OK;
}

void ygzfe_frame_destroy(ygzfe_frame *f) {
    if (!f) return;
    (void)hipSetDevice(f->ex->device);
    {
        // an alignment in flight (ygzfe_sparse_align_begin, on ex->astream) may read this
        // frame's pyramid: wait for it (its result stays staged for _end)
        std::lock_guard<std::mutex> lk(f->ex->mu);
        if (f->ex->align_pending) (void)hipEventSynchronize(f->ex->ev_align_done);
        (void)hipStreamSynchronize(f->ex->stream);
    }
    std::lock_guard<std::recursive_mutex> lk(graph_mutex());
    ygzfe_extractor *ex = f->ex;
    delete f;
    if (--ex->live_frames == 0 && ex->dead) extractor_release(ex);
}

static int pyramid_from_level0(ygzfe_frame *f, hipStream_t st) {
    const PlanDev &pd = *f->plan;
    YGZ_HIP(launch_pyramid(f->pyr.as<uint8_t>(), pd.hp().pyr_bytes, pd.hp(), pd.dp(), pd.tabs.as<int>(), 1, st));
    return YGZFE_OK;
}

int ygzfe_compute_pyramid(ygzfe_extractor *ex, ygzfe_frame *f, const uint8_t *img, int stride) {
    if (!ex || !f || !img || stride < f->W) { set_error("invalid argument"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    // the image is copied into pinned staging (the caller may reuse `img` at once)
    // and DMA'd from there; everything that reads the pyramid is ordered after it
    // on ex->stream or synchronises first (ygzfe_frame_level), so no
    // synchronisation here -- only before the staging is overwritten
    YGZ_TRY(ex->ensure_side());
    const size_t n = (size_t)f->W * f->H;
    YGZ_HIP(hipEventSynchronize(ex->ev_img));  // the previous DMA out of himg (before it may be reallocated)
    YGZ_TRY(ex->order_after_align(ex->stream));
    YGZ_TRY(ex->himg.ensure(n));
    uint8_t *h = ex->himg.as<uint8_t>();
    if (stride == f->W) {
        memcpy(h, img, n);
    } else {
        for (int y = 0; y < f->H; y++) memcpy(h + (size_t)y * f->W, img + (size_t)y * stride, (size_t)f->W);
    }
    YGZ_HIP(hipMemcpyAsync(f->pyr.p, h, n, hipMemcpyHostToDevice, ex->stream));
    YGZ_HIP(hipEventRecord(ex->ev_img, ex->stream));
    YGZ_TRY(pyramid_from_level0(f, ex->stream));
    return YGZFE_OK;
}

int ygzfe_compute_pyramid_device(ygzfe_extractor *ex, ygzfe_frame *f, const uint8_t *d_img, int stride,
                                 void *stream) {
    if (!ex || !f || !d_img || stride < f->W) { set_error("invalid argument"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(ex->device));
    hipStream_t st = stream ? (hipStream_t)stream : ex->stream;
    YGZ_TRY(ex->order_after_align(st));
    YGZ_HIP(hipMemcpy2DAsync(f->pyr.p, f->W, d_img, stride, f->W, f->H, hipMemcpyDeviceToDevice, st));
    YGZ_TRY(pyramid_from_level0(f, st));
    if (!stream) YGZ_HIP(hipStreamSynchronize(st));
    return YGZFE_OK;
}

int ygzfe_frame_level(const ygzfe_frame *f, int level, int *w, int *h, uint8_t *dst, int dst_stride) {
    if (!f) { set_error("null frame"); return YGZFE_EINVAL; }
    const Plan &P = f->plan->hp();
    if (level < 0 || level >= P.nlevels) { set_error("level %d out of range", level); return YGZFE_EINVAL; }
    const LevelDesc &L = P.lv[level];
    if (w) *w = L.w;
    if (h) *h = L.h;
    if (dst) {
        if (dst_stride < L.w) { set_error("dst_stride < level width"); return YGZFE_EINVAL; }
        ygzfe_extractor *ex = f->ex;
        YGZ_TRY(ensure_device(ex->device));
        std::lock_guard<std::mutex> lk(ex->mu);
        // one contiguous DMA into page-locked staging, ordered after the frame's work on
        // ex->stream, then the row copy on the host
        const size_t n = (size_t)L.w * L.h;
        YGZ_HIP(hipStreamSynchronize(ex->stream));  // the staging's previous use, the pyramid's writers
        YGZ_TRY(ex->hlvl.ensure(n));
        YGZ_HIP(hipMemcpyAsync(ex->hlvl.p, f->pyr.as<uint8_t>() + L.off, n, hipMemcpyDeviceToHost, ex->stream));
        YGZ_HIP(hipStreamSynchronize(ex->stream));
        const uint8_t *hs = ex->hlvl.as<uint8_t>();
        if (dst_stride == L.w) {
            memcpy(dst, hs, n);
        } else {
            for (int y = 0; y < L.h; y++) memcpy(dst + (size_t)y * dst_stride, hs + (size_t)y * L.w, (size_t)L.w);
        }
    }
    return YGZFE_OK;
}

int ygzfe_frame_set_level(ygzfe_frame *f, int level, const uint8_t *src, int src_stride) {
    if (!f || !src) { set_error("null argument"); return YGZFE_EINVAL; }
    const Plan &P = f->plan->hp();
    if (level < 0 || level >= P.nlevels) { set_error("level %d out of range", level); return YGZFE_EINVAL; }
    const LevelDesc &L = P.lv[level];
    if (src_stride < L.w) { set_error("src_stride < level width"); return YGZFE_EINVAL; }
    ygzfe_extractor *ex = f->ex;
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    YGZ_HIP(hipStreamSynchronize(ex->stream));  // the staging's previous use
    if (ex->align_pending) YGZ_HIP(hipEventSynchronize(ex->ev_align_done));  // an alignment reading this pyramid
    const size_t n = (size_t)L.w * L.h;
    YGZ_TRY(ex->hlvl.ensure(n));
    uint8_t *hs = ex->hlvl.as<uint8_t>();
    if (src_stride == L.w) {
        memcpy(hs, src, n);
    } else {
        for (int y = 0; y < L.h; y++) memcpy(hs + (size_t)y * L.w, src + (size_t)y * src_stride, (size_t)L.w);
    }
    YGZ_HIP(hipMemcpyAsync(f->pyr.as<uint8_t>() + L.off, hs, n, hipMemcpyHostToDevice, ex->stream));
    YGZ_HIP(hipStreamSynchronize(ex->stream));  // the level is in place when the call returns, as before
    return YGZFE_OK;
}

// levels [first, first + count) of the plan: checked range, and the device span
// [lv[first].off, lv[last].off + w * h) that holds them (one DMA for all)
static int level_span(const ygzfe_frame *f, int first, int count, size_t *off, size_t *bytes) {
    const Plan &P = f->plan->hp();
    if (first < 0 || count < 1 || first + count > P.nlevels) {
        set_error("levels [%d, %d) out of range (%d levels)", first, first + count, P.nlevels);
        return YGZFE_EINVAL;
    }
    const LevelDesc &a = P.lv[first], &b = P.lv[first + count - 1];
    *off = a.off;
    *bytes = (size_t)b.off + (size_t)b.w * b.h - a.off;
    return YGZFE_OK;
}

int ygzfe_frame_levels(const ygzfe_frame *f, int first, int count, uint8_t *const *dst, const int *dst_stride) {
    if (!f || !dst || !dst_stride) { set_error("null argument"); return YGZFE_EINVAL; }
    size_t off = 0, bytes = 0;
    YGZ_TRY(level_span(f, first, count, &off, &bytes));
    const Plan &P = f->plan->hp();
    for (int i = 0; i < count; i++)
        if (!dst[i] || dst_stride[i] < P.lv[first + i].w) { set_error("level %d: no buffer or stride < width", first + i); return YGZFE_EINVAL; }
    ygzfe_extractor *ex = f->ex;
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    // every level in one DMA into page-locked staging, ordered after the pyramid's writers on
    // ex->stream; one synchronisation, then the row copies on the host
    // (every user of the staging synchronises before it returns, under ex->mu)
    YGZ_TRY(ex->hlvl.ensure(bytes));
    YGZ_HIP(hipMemcpyAsync(ex->hlvl.p, f->pyr.as<uint8_t>() + off, bytes, hipMemcpyDeviceToHost, ex->stream));
    YGZ_HIP(hipStreamSynchronize(ex->stream));
    for (int i = 0; i < count; i++) {
        const LevelDesc &L = P.lv[first + i];
        const uint8_t *hs = ex->hlvl.as<uint8_t>() + (L.off - off);
        if (dst_stride[i] == L.w) {
            memcpy(dst[i], hs, (size_t)L.w * L.h);
        } else {
            for (int y = 0; y < L.h; y++) memcpy(dst[i] + (size_t)y * dst_stride[i], hs + (size_t)y * L.w, (size_t)L.w);
        }
    }
    return YGZFE_OK;
}

int ygzfe_frame_set_levels(ygzfe_frame *f, int first, int count, const uint8_t *const *src, const int *src_stride) {
    if (!f || !src || !src_stride) { set_error("null argument"); return YGZFE_EINVAL; }
    size_t off = 0, bytes = 0;
    YGZ_TRY(level_span(f, first, count, &off, &bytes));
    const Plan &P = f->plan->hp();
    for (int i = 0; i < count; i++)
        if (!src[i] || src_stride[i] < P.lv[first + i].w) { set_error("level %d: no buffer or stride < width", first + i); return YGZFE_EINVAL; }
    ygzfe_extractor *ex = f->ex;
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    if (ex->align_pending) YGZ_HIP(hipEventSynchronize(ex->ev_align_done));  // an alignment reading this pyramid
    // no DMA may still target the staging (an earlier call that returned on an error
    // between its async copy and its synchronisation), as in ygzfe_frame_set_level
    YGZ_HIP(hipStreamSynchronize(ex->stream));
    YGZ_TRY(ex->hlvl.ensure(bytes));
    for (int i = 0; i < count; i++) {
        const LevelDesc &L = P.lv[first + i];
        uint8_t *hs = ex->hlvl.as<uint8_t>() + (L.off - off);
        if (src_stride[i] == L.w) {
            memcpy(hs, src[i], (size_t)L.w * L.h);
        } else {
            for (int y = 0; y < L.h; y++) memcpy(hs + (size_t)y * L.w, src[i] + (size_t)y * src_stride[i], (size_t)L.w);
        }
    }
    // the gaps between levels carry staging bytes: no kernel reads them as pixels
    YGZ_HIP(hipMemcpyAsync(f->pyr.as<uint8_t>() + off, ex->hlvl.p, bytes, hipMemcpyHostToDevice, ex->stream));
    YGZ_HIP(hipStreamSynchronize(ex->stream));  // the levels are in place when the call returns
    return YGZFE_OK;
}

static int dso_max_rows(const Plan &P) {
    const int g = 7;
    return 3 * (P.lv[0].w / g) * (P.lv[0].h / g);
}

// YGZFE_TRACE=1 (debugging): ygzfe_extract's steps on stderr
static void trace_step(const char *what, long a = 0, long b = 0) {
    static const bool on = getenv("YGZFE_TRACE") != nullptr;
    if (on) {
        fprintf(stderr, "[ygzfe_extract] %s %ld %ld\n", what, a, b);
        fflush(stderr);
    }
}

int ygzfe_extract(ygzfe_extractor *ex, ygzfe_frame *f, int method, ygzfe_kp *kps_io, int n_existing, int cap,
                  uint8_t *desc, int *n_out) {
    trace_step("enter", method, cap);
    if (!ex || !f || !n_out || n_existing < 0 || (n_existing > 0 && !kps_io)) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (method == YGZFE_FAST_KEYPOINT) {
        set_error("FAST_KEYPOINT is flagged buggy and never called by the reference (ORBextractor.cc:1191)");
        return YGZFE_EINVAL;
    }
    if (method != YGZFE_ORBSLAM_KEYPOINT && method != YGZFE_DSO_KEYPOINT) {
        set_error("unknown method %d", method);
        return YGZFE_EINVAL;
    }
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    const PlanDev &pd = *f->plan;
    const Plan &P = pd.hp();
    hipStream_t st = ex->stream;
    const int rows = n_existing + (method == YGZFE_DSO_KEYPOINT ? std::max(P.kp_cap, dso_max_rows(P)) : P.kp_cap);
    Workspace &ws = ex->ws;
    YGZ_TRY(ws.ensure(P, 1, rows));
    trace_step("workspace", rows, P.kp_cap);
    const uint8_t *pyr = f->pyr.as<uint8_t>();
    int total = 0;
    if (method == YGZFE_ORBSLAM_KEYPOINT) {
        // The single-frame DAG (one Tracking thread's latency): the blur on side[0]
        // beside FAST (st); the octree on st (its node-pool classes in sequence, or with
        // YGZFE_OCT_FORK the classes after the first on side[1]); keypoint rows, angle +
        // rBRIEF after the blur's join; one packing kernel, one D2H into pinned memory,
        // one synchronisation.  Every stream forked here is joined back into st before
        // the capture ends (checked after every capture).
        YGZ_TRY(ex->ensure_side());
        // The rows, descriptors, count and octree-overflow flag are written straight
        // into one result buffer -- [count, flag, 0, 0][rows x 28 B keypoints]
        // [16-B aligned: rows x 32 B descriptors] -- so one D2H returns everything.
        const size_t kbytes = align16(sizeof(ygzfe_kp) * (size_t)rows), rbytes = 16 + kbytes + (size_t)32 * rows;
        YGZ_TRY(ex->res.ensure(rbytes));
        YGZ_TRY(ex->hout.ensure(rbytes));
        uint8_t *res = ex->res.as<uint8_t>();
        int *d_count = reinterpret_cast<int *>(res), *d_err = d_count + 1;
        ygzfe_kp *d_kps = reinterpret_cast<ygzfe_kp *>(res + 16);
        uint8_t *d_desc = res + 16 + kbytes;
        const int *d_nexist = nullptr;  // null: no existing rows (the kernels read 0)
        if (n_existing > 0) {
            YGZ_TRY(ex->hin.ensure(16 + sizeof(ygzfe_kp) * (size_t)n_existing));
            ex->hin.as<int>()[0] = n_existing;
            memcpy(ex->hin.as<uint8_t>() + 16, kps_io, sizeof(ygzfe_kp) * n_existing);
            YGZ_HIP(hipMemcpyAsync(ws.nexist.p, ex->hin.p, sizeof(int), hipMemcpyHostToDevice, st));
            YGZ_HIP(hipMemcpyAsync(d_kps, ex->hin.as<uint8_t>() + 16, sizeof(ygzfe_kp) * n_existing,
                                   hipMemcpyHostToDevice, st));
            d_nexist = ws.nexist.as<int>();
        }
        // the header and, speculatively, as many rows as the caller can take (one DMA)
        const int cap_rows = std::min(rows, std::max(cap, 0));
        const size_t copy = desc ? 16 + kbytes + (size_t)32 * cap_rows : 16 + sizeof(ygzfe_kp) * (size_t)cap_rows;
        hipStream_t *sd = ex->side;
        // the DAG: blur on side[0] beside FAST (every level in one launch; its first
        // lane also clears the overflow flag) on st; the octree; rows + jobs, then
        // angle + rBRIEF after the blur joins; the D2H.  Only side[0] waits on ev_fork:
        // round 5 forked all three side streams here and joined only side[0], and a
        // capture of that crashed inside hipGraphLaunch (profiles/r05_graph_fork.txt).
        static const bool oct_fork = getenv("YGZFE_OCT_FORK") != nullptr;
        auto enqueue = [&]() -> int {
            YGZ_HIP(hipEventRecord(ex->ev_fork, st));
            YGZ_HIP(hipStreamWaitEvent(sd[0], ex->ev_fork, 0));
            YGZ_HIP(launch_blur(pyr, ws.blur.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), 1, sd[0]));
            YGZ_HIP(hipEventRecord(ex->ev_join[0], sd[0]));
            YGZ_HIP(launch_fast_merged(pyr, P.pyr_bytes, P, pd.dp(), pd.cells.as<CellDesc>(),
                                       ws.cellbuf.as<uint32_t>(), ws.cellcnt.as<int>(), 1, st, d_err));
            // the node-pool classes (nfeatures > ~1000 puts level 0 in a larger class than
            // the rest): in sequence on st, or forked onto side[1] (launch_octree records
            // its own fork event after FAST and joins side[1] back before it returns)
            YGZ_HIP(launch_octree(P, pd.dp(), ws.cellbuf.as<uint32_t>(), ws.cellcnt.as<int>(), ws.candA.as<uint32_t>(),
                                  ws.candB.as<uint32_t>(), ws.sel.as<uint32_t>(), ws.selcnt.as<int>(), d_err,
                                  ws.octq.as<int>(), 1, st, oct_fork ? &sd[1] : nullptr, oct_fork ? 1 : 0,
                                  ex->ev_oct_fork, ex->ev_oct_join, true));
            YGZ_HIP(launch_emit_kps(P, pd.dp(), ws.sel.as<uint32_t>(), ws.selcnt.as<int>(), d_nexist, d_kps, d_count,
                                    rows, ws.ojobs.as<uint2>(), 1, st));
            YGZ_HIP(hipStreamWaitEvent(st, ex->ev_join[0], 0));  // the blurred levels
            YGZ_HIP(launch_orient_desc(pyr, ws.blur.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), ws.ojobs.as<uint2>(),
                                       d_nexist, d_kps, d_desc, rows, 1, st));
            YGZ_HIP(launch_desc_existing(pyr, ws.blur.as<uint8_t>(), pd.dp(), d_kps, d_desc, n_existing, 0, st));
            YGZ_HIP(hipMemcpyAsync(ex->hout.p, res, copy, hipMemcpyDeviceToHost, st));
            return YGZFE_OK;
        };
        // Without existing rows the whole sequence (9-12 launches, the event fork /
        // joins and the D2H) is replayed from a HIP graph captured once per frame
        // handle: one submission instead of one host call per launch.  The graph is
        // re-captured when any buffer it names has moved or the copy size changed.
        const void *key[15] = {pyr,          ws.blur.p,  ws.cellbuf.p, ws.sel.p,       ws.candA.p,
                               ws.candB.p,   ex->res.p,  ex->hout.p,   ws.ojobs.p,     ws.cellcnt.p,
                               ws.selcnt.p,  pd.cells.p, pd.plan.p,    pd.tabs.p,      ws.octq.p};
        static_assert(sizeof(key) == sizeof(f->gkey), "graph key size");
        static const bool no_graph = getenv("YGZFE_NO_GRAPH") != nullptr;
        bool launched = false;
        trace_step("staged", (long)rbytes, (long)copy);
        if (n_existing == 0 && !no_graph && !ex->graph_broken) {
            if (!f->gexec || memcmp(f->gkey, key, sizeof(key)) != 0 || f->grows != rows || f->gcopy != copy) {
                trace_step("capture", (long)(f->gexec != nullptr), 0);
                std::lock_guard<std::recursive_mutex> lk(graph_mutex());
                f->drop_graph();
                bool ok = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) == hipSuccess;
                const int rc = ok ? enqueue() : YGZFE_EHIP;
                hipGraph_t g = nullptr;
                if (ok) ok = hipStreamEndCapture(st, &g) == hipSuccess && rc == YGZFE_OK && g;
                f->graph = g;
                // a stream still capturing after the origin's EndCapture is an unjoined fork:
                // its next launch would land in this graph, freed by the next drop_graph()
                const int bad = ex->capture_left_open();
                if (bad >= 0) {
                    f->drop_graph();
                    ex->graph_broken = true;
                    (void)hipGetLastError();
                    set_error("stream %d still capturing after ygzfe_extract's capture ended", bad);
                    return YGZFE_EHIP;
                }
                if (ok) ok = hipGraphInstantiate(&f->gexec, g, nullptr, nullptr, 0) == hipSuccess;
                if (ok) {
                    memcpy(f->gkey, key, sizeof(key));
                    f->grows = rows;
                    f->gcopy = copy;
                } else {  // capture unsupported here: plain launches from now on
                    f->drop_graph();
                    ex->graph_broken = true;
                    (void)hipGetLastError();
                }
            }
            if (f->gexec) {
                YGZ_HIP(hipGraphLaunch(f->gexec, st));
                launched = true;
            }
        }
        trace_step("launched", launched, 0);
        if (!launched) YGZ_TRY(enqueue());
        YGZ_HIP(hipStreamSynchronize(st));
        total = ex->hout.as<int>()[0];
        trace_step("synced", total, ex->hout.as<int>()[1]);
        if (ex->hout.as<int>()[1]) {
            set_error("octree node pool overflow");
            return YGZFE_EINVAL;
        }
        *n_out = total;
        if (total > cap) {
            set_error("capacity %d < %d keypoints", cap, total);
            return YGZFE_ECAP;
        }
        if (total > 0) {
            memcpy(kps_io, ex->hout.as<uint8_t>() + 16, sizeof(ygzfe_kp) * (size_t)total);
            if (desc) memcpy(desc, ex->hout.as<uint8_t>() + 16 + kbytes, (size_t)32 * total);
        }
        return YGZFE_OK;
    } else {
        if (n_existing > 0)
            YGZ_HIP(hipMemcpyAsync(ws.kps.p, kps_io, sizeof(ygzfe_kp) * n_existing, hipMemcpyHostToDevice, st));
        YGZ_HIP(launch_blur(pyr, ws.blur.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), 1, st));
        // DSO_KEYPOINT: ComputeKeyPointsDSOSingleLevel (ORBextractor.cc:1275-1386)
        const LevelDesc &L0 = P.lv[0];
        const int w = L0.w, h = L0.h, n = ex->p.nfeatures;
        YGZ_TRY(ws.occ.ensure((size_t)w * h));
        YGZ_HIP(launch_dso_occupancy(ws.kps.as<ygzfe_kp>(), n_existing, ws.occ.as<uint8_t>(), w, h, st));
        int g = ex->dso_grid;
        if (g < 0) g = (int)sqrt(1.0 * h * w / (n > 0 ? n : 1));
        int cnt = 0;
        for (;;) {
            if (cnt >= n) break;
            if (cnt > 0) {
                g -= 5;
                if (g < 7) { g = 7; break; }
            }
            if (g > kDsoMaxGridHost) {
                set_error("DSO grid %d exceeds the supported %d", g, kDsoMaxGridHost);
                return YGZFE_EINVAL;
            }
            const int ncells = (h / g) * (w / g);
            YGZ_TRY(ws.dso_keys.ensure((size_t)ncells * 3 * 4 + 16));
            YGZ_TRY(ws.dso_cnt.ensure((size_t)ncells * 4 + 16));
            YGZ_TRY(ws.dso_total.ensure(16));
            YGZ_HIP(launch_dso_pass(pyr, w, h, g, ws.occ.as<uint8_t>(), ws.dso_keys.as<uint32_t>(),
                                    ws.dso_cnt.as<int>(), st));
            YGZ_HIP(launch_dso_finish2(ws.dso_keys.as<uint32_t>(), ws.dso_cnt.as<int>(), ncells,
                                       ws.kps.as<ygzfe_kp>(), n_existing, ws.dso_total.as<int>(), st));
            YGZ_HIP(hipMemcpyAsync(&cnt, ws.dso_total.p, sizeof(int), hipMemcpyDeviceToHost, st));
            YGZ_HIP(hipStreamSynchronize(st));
            if (cnt == 0) break;  // the reference loops forever on a corner-free image
        }
        if (cnt > n) g += 5;
        ex->dso_grid = g;
        total = n_existing + cnt;
        YGZ_HIP(launch_desc_existing(pyr, ws.blur.as<uint8_t>(), pd.dp(), ws.kps.as<ygzfe_kp>(),
                                     ws.desc.as<uint8_t>(), total, 1, st));
        YGZ_HIP(hipStreamSynchronize(st));
    }
    *n_out = total;
    if (total > cap) {
        set_error("capacity %d < %d keypoints", cap, total);
        return YGZFE_ECAP;
    }
    if (total > 0) {
        YGZ_HIP(hipMemcpyAsync(kps_io, ws.kps.p, sizeof(ygzfe_kp) * total, hipMemcpyDeviceToHost, st));
        if (desc) YGZ_HIP(hipMemcpyAsync(desc, ws.desc.p, (size_t)32 * total, hipMemcpyDeviceToHost, st));
        YGZ_HIP(hipStreamSynchronize(st));
    }
    return YGZFE_OK;
}

int ygzfe_detect_and_compute(ygzfe_extractor *ex, ygzfe_frame *f, const uint8_t *img, int stride, ygzfe_kp *kps,
                             int cap, uint8_t *desc, int *n_out) {
    if (!img) { set_error("empty image"); return YGZFE_EINVAL; }  // reference returns silently (:972-973)
    YGZ_TRY(ygzfe_compute_pyramid(ex, f, img, stride));
    return ygzfe_extract(ex, f, YGZFE_ORBSLAM_KEYPOINT, kps, 0, cap, desc, n_out);
}

// ------------------------------------------------------------------ batch
int ygzfe_batch_create(const ygzfe_orb_params *p, int device, int width, int height, int max_frames,
                       ygzfe_batch **out) {
    if (!p || !out || max_frames <= 0) { set_error("invalid argument"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(device));
    std::unique_ptr<ygzfe_batch> b(new ygzfe_batch());
    b->p = *p;
    b->device = device;
    b->maxF = max_frames;
    YGZ_TRY(make_plan(*p, width, height, &b->plan));
    const Plan &P = b->plan->hp();
    YGZ_TRY(b->pyr.ensure((size_t)max_frames * P.pyr_bytes));
    YGZ_TRY(b->ws.ensure(P, max_frames, P.kp_cap));
    YGZ_HIP(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
    for (int i = 0; i < 3; i++) {
        YGZ_HIP(hipStreamCreateWithFlags(&b->aux[i], hipStreamNonBlocking));
        YGZ_HIP(hipEventCreateWithFlags(&b->ev_join[i], hipEventDisableTiming));
    }
    YGZ_HIP(hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming));
    YGZ_HIP(hipEventCreateWithFlags(&b->ev_oct_fork, hipEventDisableTiming));
    YGZ_HIP(hipEventCreateWithFlags(&b->ev_desc_done, hipEventDisableTiming));
    for (int i = 0; i < 2; i++) YGZ_HIP(hipEventCreateWithFlags(&b->ev_oct_join[i], hipEventDisableTiming));
    *out = b.release();
    return YGZFE_OK;
}

void ygzfe_batch_destroy(ygzfe_batch *b) {
    if (!b) return;
    std::lock_guard<std::recursive_mutex> lk(graph_mutex());
    (void)hipSetDevice(b->device);
    (void)hipStreamSynchronize(b->stream);
    (void)b->collect();
    for (auto &e : b->pool) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(b->stream);
    for (int i = 0; i < 3; i++) {
        if (b->aux[i]) (void)hipStreamSynchronize(b->aux[i]), (void)hipStreamDestroy(b->aux[i]);
        if (b->ev_join[i]) (void)hipEventDestroy(b->ev_join[i]);
    }
    if (b->ev_fork) (void)hipEventDestroy(b->ev_fork);
    if (b->ev_oct_fork) (void)hipEventDestroy(b->ev_oct_fork);
    if (b->ev_desc_done) (void)hipEventSynchronize(b->ev_desc_done), (void)hipEventDestroy(b->ev_desc_done);
    for (int i = 0; i < 2; i++)
        if (b->ev_oct_join[i]) (void)hipEventDestroy(b->ev_oct_join[i]);
    delete b;
}

int ygzfe_batch_info(ygzfe_batch *b, size_t *frame_pitch, int *kp_cap, int *nlevels) {
    if (!b) { set_error("null batch"); return YGZFE_EINVAL; }
    const Plan &P = b->plan->hp();
    if (frame_pitch) *frame_pitch = P.pyr_bytes;
    if (kp_cap) *kp_cap = P.kp_cap;
    if (nlevels) *nlevels = P.nlevels;
    return YGZFE_OK;
}

int ygzfe_batch_frames(ygzfe_batch *b, uint8_t **d_frames) {
    if (!b || !d_frames) { set_error("null argument"); return YGZFE_EINVAL; }
    *d_frames = b->pyr.as<uint8_t>();
    return YGZFE_OK;
}

int ygzfe_batch_bind_buffers(ygzfe_batch *b, uint8_t *d_pyramids, ygzfe_kp *d_kps, uint8_t *d_desc,
                             int32_t *d_counts) {
    if (!b) { set_error("null batch"); return YGZFE_EINVAL; }
    const Plan &P = b->plan->hp();
    YGZ_TRY(ensure_device(b->device));
    YGZ_HIP(hipStreamSynchronize(b->stream));
    if (d_pyramids) b->pyr.bind(d_pyramids, (size_t)b->maxF * P.pyr_bytes);
    if (d_kps) b->ws.kps.bind(d_kps, (size_t)b->maxF * P.kp_cap * sizeof(ygzfe_kp));
    if (d_desc) b->ws.desc.bind(d_desc, (size_t)b->maxF * P.kp_cap * 32);
    if (d_counts) b->ws.counts.bind(d_counts, (size_t)b->maxF * 4);
    return YGZFE_OK;
}

int ygzfe_batch_upload(ygzfe_batch *b, const uint8_t *frames, int n_frames) {
    if (!b || !frames || n_frames < 0 || n_frames > b->maxF) { set_error("invalid argument"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(b->device));
    const Plan &P = b->plan->hp();
    // the previous extraction (possibly on caller streams) may still read the slots
    if (b->desc_pending) YGZ_HIP(hipStreamWaitEvent(b->stream, b->ev_desc_done, 0));
    // frame i -> level-0 slot of pyramid i (pitch P.pyr_bytes)
    YGZ_HIP(hipMemcpy2DAsync(b->pyr.p, P.pyr_bytes, frames, (size_t)P.W * P.H, (size_t)P.W * P.H, n_frames,
                             hipMemcpyHostToDevice, b->stream));
    YGZ_HIP(hipStreamSynchronize(b->stream));
    return YGZFE_OK;
}

// Extraction as a small DAG over the launch stream and two helpers:
//   kp_stream:   pyramid -> FAST levels -> octree -> keypoint rows
//   desc_stream: (after the pyramid) GaussianBlur, concurrent with FAST;
//                (after the keypoint rows) angle + rBRIEF
// Work queued on kp_stream afterwards sees the keypoint rows (positions,
// octave, size, response; not the angle); work on desc_stream sees the
// complete rows and descriptors.
int ygzfe_batch_extract_split(ygzfe_batch *b, int n_frames, void *kp_stream, void *desc_stream) {
    if (!b || n_frames < 0 || n_frames > b->maxF) { set_error("invalid argument"); return YGZFE_EINVAL; }
    if (n_frames == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(b->device));
    hipStream_t st = kp_stream ? (hipStream_t)kp_stream : b->stream;
    hipStream_t ds = desc_stream ? (hipStream_t)desc_stream : st;
    const PlanDev &pd = *b->plan;
    const Plan &P = pd.hp();
    Workspace &ws = b->ws;
    uint8_t *pyr = b->pyr.as<uint8_t>();
    // write-after-read across calls: the previous call's descriptor pass (on its
    // desc_stream) still reads the pyramid, blur and octree selection this call rewrites
    // (not while capturing a graph: a replay retires as a whole before the next)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    YGZ_HIP(hipStreamIsCapturing(st, &cap));
    if (b->desc_pending && cap == hipStreamCaptureStatusNone) YGZ_HIP(hipStreamWaitEvent(st, b->ev_desc_done, 0));
    YGZ_HIP(hipMemsetAsync(ws.err.p, 0, 16, st));
    // An all-area pyramid (C2: levels 1..3 exact x2 INTER_AREA) is formed by the level-0
    // blur strips as they stream level 0 (k_blur7's fused mode: level 0 read once for both),
    // on st before FAST; the other levels' blur then goes beside FAST.  (Timed as the
    // pyramid stage; YGZFE_PYR_UNFUSED=1 keeps the separate pyramid pass, for A/B.)
    static const bool unfused = getenv("YGZFE_PYR_UNFUSED") != nullptr;
    const bool fused = !unfused && pyramid_fusable(P) > 0;
    hipEvent_t t0 = b->begin(st);
    if (fused)
        YGZ_HIP(launch_pyramid_blur0(pyr, ws.blur.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), n_frames, st));
    else
        YGZ_HIP(launch_pyramid(pyr, P.pyr_bytes, P, pd.dp(), pd.tabs.as<int>(), n_frames, st));
    b->end(ST_PYR, t0, st);
    // the blur feeds only the descriptors: on desc_stream, beside FAST.  (Both
    // are VALU-bound; beside the octree instead, the blur slows the octree's
    // latency-bound passes by as much as it would slow FAST.)  A separate
    // stream of ygzfe's own may share the caller's hardware queue.
    hipStream_t bs = ds;
    if (ds != st) {
        YGZ_HIP(hipEventRecord(b->ev_fork, st));
        YGZ_HIP(hipStreamWaitEvent(ds, b->ev_fork, 0));
    }
    t0 = b->begin(bs);
    if (fused)
        YGZ_HIP(launch_blur_rest(pyr, ws.blur.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), n_frames, bs));
    else
        YGZ_HIP(launch_blur(pyr, ws.blur.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), n_frames, bs));
    b->end(ST_BLUR, t0, bs);
    t0 = b->begin(st);
    YGZ_HIP(launch_fast(pyr, P.pyr_bytes, P, pd.dp(), pd.cells.as<CellDesc>(), ws.cellbuf.as<uint32_t>(),
                        ws.cellcnt.as<int>(), n_frames, st));
    b->end(ST_FAST, t0, st);
    t0 = b->begin(st);
    YGZ_HIP(launch_octree(P, pd.dp(), ws.cellbuf.as<uint32_t>(), ws.cellcnt.as<int>(), ws.candA.as<uint32_t>(),
                          ws.candB.as<uint32_t>(), ws.sel.as<uint32_t>(), ws.selcnt.as<int>(), ws.err.as<int>(),
                          ws.octq.as<int>(),
                          n_frames, st, &b->aux[1], 2, b->ev_oct_fork, b->ev_oct_join));
    YGZ_HIP(launch_emit_kps(P, pd.dp(), ws.sel.as<uint32_t>(), ws.selcnt.as<int>(), nullptr, ws.kps.as<ygzfe_kp>(),
                            ws.counts.as<int>(), P.kp_cap, ws.ojobs.as<uint2>(), n_frames, st));
    b->end(ST_OCT, t0, st);
    // descriptors: after the blur (already on ds) and the keypoint rows
    if (ds != st) {
        YGZ_HIP(hipEventRecord(b->ev_join[1], st));
        YGZ_HIP(hipStreamWaitEvent(ds, b->ev_join[1], 0));
    }
    t0 = b->begin(ds);
    YGZ_HIP(launch_orient_desc(pyr, ws.blur.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), ws.ojobs.as<uint2>(), nullptr,
                               ws.kps.as<ygzfe_kp>(), ws.desc.as<uint8_t>(), P.kp_cap, n_frames, ds));
    b->end(ST_DESC, t0, ds);
    if (cap == hipStreamCaptureStatusNone) {
        YGZ_HIP(hipEventRecord(b->ev_desc_done, ds));
        b->desc_pending = true;
    }
    return YGZFE_OK;
}

int ygzfe_batch_extract(ygzfe_batch *b, int n_frames, void *stream) {
    // everything complete on `stream` when the last launch retires
    return ygzfe_batch_extract_split(b, n_frames, stream, stream);
}

// Measurement helper (tools/mb_fast.py): one stage alone over the first n_frames
// resident frames, `reps` back-to-back launch sets on the batch stream, average
// ms per set (hipEvents).  stage 0: FAST (writes only the cell scratch; pyramid
// levels built first when build_pyramid); stage 1: orientation + rBRIEF on the
// octree selection of the last full extraction (rewrites its angles and descriptors);
// stage 2: the GaussianBlur of every level.
int ygzfe_diag_stage_ms(ygzfe_batch *b, int stage, int n_frames, int reps, int build_pyramid, float *ms) {
    if (!b || !ms || n_frames < 1 || n_frames > b->maxF || reps < 1 || stage < 0 || stage > 2) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    YGZ_TRY(ensure_device(b->device));
    const PlanDev &pd = *b->plan;
    const Plan &P = pd.hp();
    const uint8_t *pyr = b->pyr.as<uint8_t>();
    if (build_pyramid)
        YGZ_HIP(launch_pyramid(b->pyr.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), pd.tabs.as<int>(), n_frames, b->stream));
    hipEvent_t e0, e1;
    YGZ_HIP(hipEventCreate(&e0));
    YGZ_HIP(hipEventCreate(&e1));
    YGZ_HIP(hipEventRecord(e0, b->stream));
    Workspace &ws = b->ws;
    for (int r = 0; r < reps; r++) {
        if (stage == 0)
            YGZ_HIP(launch_fast(pyr, P.pyr_bytes, P, pd.dp(), pd.cells.as<CellDesc>(), ws.cellbuf.as<uint32_t>(),
                                ws.cellcnt.as<int>(), n_frames, b->stream));
        else if (stage == 2)
            YGZ_HIP(launch_blur(pyr, ws.blur.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), n_frames, b->stream));
        else
            YGZ_HIP(launch_orient_desc(pyr, ws.blur.as<uint8_t>(), P.pyr_bytes, P, pd.dp(), ws.ojobs.as<uint2>(),
                                       nullptr, ws.kps.as<ygzfe_kp>(), ws.desc.as<uint8_t>(), P.kp_cap, n_frames,
                                       b->stream));
    }
    YGZ_HIP(hipEventRecord(e1, b->stream));
    YGZ_HIP(hipEventSynchronize(e1));
    YGZ_HIP(hipEventElapsedTime(ms, e0, e1));
    *ms /= reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return YGZFE_OK;
}

// Host reads of extraction outputs: the batch stream (uploads, own launches) and the
// last extraction's end event (its descriptor pass, after every other stage joined)
// instead of a device-wide synchronisation that would also wait for unrelated streams.
// An extraction captured into a caller's graph is the caller's to synchronise.
static int batch_wait(ygzfe_batch *b) {
    YGZ_HIP(hipStreamSynchronize(b->stream));
    if (b->desc_pending) YGZ_HIP(hipEventSynchronize(b->ev_desc_done));
    return YGZFE_OK;
}

int ygzfe_batch_check(ygzfe_batch *b) {
    if (!b) { set_error("null batch"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(b->device));
    int herr = 0;
    YGZ_TRY(batch_wait(b));
    YGZ_HIP(hipMemcpy(&herr, b->ws.err.p, sizeof(int), hipMemcpyDeviceToHost));
    if (herr) { set_error("octree node pool overflow"); return YGZFE_EINVAL; }
    return YGZFE_OK;
}

int ygzfe_batch_result(ygzfe_batch *b, int frame, ygzfe_kp *kps, int cap, uint8_t *desc, int *n_out) {
    if (!b || frame < 0 || frame >= b->maxF || !n_out) { set_error("invalid argument"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(b->device));
    YGZ_TRY(batch_wait(b));
    const Plan &P = b->plan->hp();
    int n = 0;
    YGZ_HIP(hipMemcpy(&n, b->ws.counts.as<int>() + frame, sizeof(int), hipMemcpyDeviceToHost));
    *n_out = n;
    if (n > cap) { set_error("capacity %d < %d", cap, n); return YGZFE_ECAP; }
    if (kps && n) YGZ_HIP(hipMemcpy(kps, b->ws.kps.as<ygzfe_kp>() + (size_t)frame * P.kp_cap, sizeof(ygzfe_kp) * n,
                                    hipMemcpyDeviceToHost));
    if (desc && n) YGZ_HIP(hipMemcpy(desc, b->ws.desc.as<uint8_t>() + (size_t)frame * P.kp_cap * 32, (size_t)32 * n,
                                     hipMemcpyDeviceToHost));
    return YGZFE_OK;
}

int ygzfe_batch_device_results(ygzfe_batch *b, ygzfe_kp **d_kps, uint8_t **d_desc, int32_t **d_counts,
                               int *kp_cap) {
    if (!b) { set_error("null batch"); return YGZFE_EINVAL; }
    if (d_kps) *d_kps = b->ws.kps.as<ygzfe_kp>();
    if (d_desc) *d_desc = b->ws.desc.as<uint8_t>();
    if (d_counts) *d_counts = b->ws.counts.as<int32_t>();
    if (kp_cap) *kp_cap = b->plan->hp().kp_cap;
    return YGZFE_OK;
}

int ygzfe_batch_level(ygzfe_batch *b, int frame, int level, const uint8_t **d_level, int *w, int *h, int *stride) {
    if (!b || frame < 0 || frame >= b->maxF) { set_error("invalid argument"); return YGZFE_EINVAL; }
    const Plan &P = b->plan->hp();
    if (level < 0 || level >= P.nlevels) { set_error("level out of range"); return YGZFE_EINVAL; }
    if (d_level) *d_level = b->pyr.as<uint8_t>() + (size_t)frame * P.pyr_bytes + P.lv[level].off;
    if (w) *w = P.lv[level].w;
    if (h) *h = P.lv[level].h;
    if (stride) *stride = P.lv[level].w;
    return YGZFE_OK;
}

int ygzfe_batch_read_level(ygzfe_batch *b, int frame, int level, int blurred, uint8_t *dst, int dst_stride) {
    if (!b || !dst || frame < 0 || frame >= b->maxF) { set_error("invalid argument"); return YGZFE_EINVAL; }
    const Plan &P = b->plan->hp();
    if (level < 0 || level >= P.nlevels) { set_error("level out of range"); return YGZFE_EINVAL; }
    const LevelDesc &L = P.lv[level];
    if (dst_stride < L.w) { set_error("dst_stride < level width"); return YGZFE_EINVAL; }
    const DevBuf &src = blurred ? b->ws.blur : b->pyr;
    if (!src.p) { set_error("no %s buffer yet (run ygzfe_batch_extract first)", blurred ? "blurred" : "pyramid"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(b->device));
    YGZ_TRY(batch_wait(b));  // extract may have run on a caller stream + side streams
    YGZ_HIP(hipMemcpy2D(dst, dst_stride, (const uint8_t *)src.p + (size_t)frame * P.pyr_bytes + L.off, L.w, L.w, L.h,
                        hipMemcpyDeviceToHost));
    return YGZFE_OK;
}

int ygzfe_batch_stats(ygzfe_batch *b, int n_frames, int64_t *candidates, int64_t *selected) {
    if (!b || n_frames < 0 || n_frames > b->maxF) { set_error("invalid argument"); return YGZFE_EINVAL; }
    const Plan &P = b->plan->hp();
    YGZ_TRY(ensure_device(b->device));
    YGZ_TRY(batch_wait(b));  // extract may have run on a caller stream + side streams
    for (int l = 0; l < P.nlevels; l++) {
        if (candidates) candidates[l] = 0;
        if (selected) selected[l] = 0;
    }
    if (n_frames == 0 || !b->ws.cellcnt.p) return YGZFE_OK;
    std::vector<int> cc((size_t)n_frames * P.ncells), sc((size_t)n_frames * P.nlevels);
    if (P.ncells) YGZ_HIP(hipMemcpy(cc.data(), b->ws.cellcnt.p, cc.size() * 4, hipMemcpyDeviceToHost));
    YGZ_HIP(hipMemcpy(sc.data(), b->ws.selcnt.p, sc.size() * 4, hipMemcpyDeviceToHost));
    for (int f = 0; f < n_frames; f++)
        for (int l = 0; l < P.nlevels; l++) {
            const LevelDesc &L = P.lv[l];
            if (candidates)
                for (int c = 0; c < L.ncells; c++) candidates[l] += cc[(size_t)f * P.ncells + L.cell_begin + c];
            if (selected) selected[l] += sc[(size_t)f * P.nlevels + l];
        }
    return YGZFE_OK;
}

int ygzfe_batch_timing(ygzfe_batch *b, int enable, float *ms, const char **names, int cap) {
    if (!b) { set_error("null batch"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(b->device));
    YGZ_TRY(b->collect());
    for (int s = 0; s < kNumStages && s < cap; s++) {
        if (ms) ms[s] = b->calls[s] ? (float)(b->total_ms[s] / b->calls[s]) : 0.f;
        if (names) names[s] = kStageNames[s];
    }
    if (enable > 0) {  // reset + enable
        for (int s = 0; s < kNumStages; s++) { b->total_ms[s] = 0; b->calls[s] = 0; }
        b->timing = true;
    } else if (enable == 0) {
        b->timing = false;
    }
    return kNumStages;
}

void *ygzfe_batch_stream(ygzfe_batch *b) { return b ? (void *)b->stream : nullptr; }

size_t ygzfe_slot_bytes(int kp_cap) {
    if (kp_cap < 0) return 0;
    return ((size_t)YGZFE_SLOT_HEADER + (size_t)kp_cap * 60 + 15) & ~(size_t)15;
}

int ygzfe_batch_pack_slots(ygzfe_batch *b, int frame_begin, int n_frames, const struct ygzfe_align_result *d_align,
                           int global_first, uint8_t *d_slots, size_t slot_pitch, void *stream) {
    if (!b || frame_begin < 0 || n_frames < 0 || frame_begin + n_frames > b->maxF || (n_frames > 0 && !d_slots)) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    const Plan &P = b->plan->hp();
    if (slot_pitch < ygzfe_slot_bytes(P.kp_cap) || (slot_pitch & 15) || ((uintptr_t)d_slots & 15)) {
        set_error("slot pitch %zu (need >= %zu, 16-B multiple, 16-B aligned base)", slot_pitch,
                  ygzfe_slot_bytes(P.kp_cap));
        return YGZFE_EINVAL;
    }
    YGZ_TRY(ensure_device(b->device));
    hipStream_t st = stream ? (hipStream_t)stream : b->stream;
    hipEvent_t t0 = b->begin(st);
    YGZ_HIP(launch_pack_slots(b->ws.kps.as<ygzfe_kp>(), b->ws.desc.as<uint8_t>(), b->ws.counts.as<int>(), P.kp_cap,
                              d_align, frame_begin, n_frames, global_first, d_slots, slot_pitch, st));
    b->end(ST_PACK, t0, st);
    return YGZFE_OK;
}

// ------------------------------------------------------------------ hamming
int ygzfe_hamming_best2_device(const uint8_t *d_query, int nq, const uint8_t *d_train, int nt, int32_t *d_best_idx,
                               int32_t *d_best_dist, int32_t *d_second_dist, void *stream) {
    if (nq < 0 || nt < 0 || (nq > 0 && (!d_query || !d_best_idx || !d_best_dist || !d_second_dist)) ||
        (nt > 0 && !d_train)) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    YGZ_HIP(launch_hamming_best2(d_query, nq, d_train, nt, d_best_idx, d_best_dist, d_second_dist,
                                 (hipStream_t)stream));
    return YGZFE_OK;
}

int ygzfe_hamming_best2(int device, const uint8_t *query, int nq, const uint8_t *train, int nt, int32_t *best_idx,
                        int32_t *best_dist, int32_t *second_dist) {
    if (nq < 0 || nt < 0 || (nq > 0 && (!query || !best_idx || !best_dist || !second_dist)) || (nt > 0 && !train)) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (nq == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(device));
    StagingLease S;
    YGZ_TRY(S.acquire(device));
    // in: [query][train]  out: [best_idx][best_dist][second_dist]
    const size_t o_t = align16((size_t)nq * 32), in_bytes = o_t + align16((size_t)(nt > 0 ? nt : 1) * 32);
    const size_t out_bytes = (size_t)nq * 12;
    YGZ_TRY(S->hin.ensure(in_bytes));
    YGZ_TRY(S->hout.ensure(out_bytes));
    YGZ_TRY(S->dev.ensure(in_bytes + out_bytes));
    uint8_t *h = S->hin.as<uint8_t>(), *d = S->dev.as<uint8_t>();
    memcpy(h, query, (size_t)nq * 32);
    if (nt > 0) memcpy(h + o_t, train, (size_t)nt * 32);
    YGZ_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, S->stream));
    int32_t *bi = reinterpret_cast<int32_t *>(d + in_bytes), *bd = bi + nq, *sd = bd + nq;
    YGZ_HIP(launch_hamming_best2(d, nq, d + o_t, nt, bi, bd, sd, S->stream));
    YGZ_HIP(hipMemcpyAsync(S->hout.p, bi, out_bytes, hipMemcpyDeviceToHost, S->stream));
    YGZ_HIP(hipStreamSynchronize(S->stream));
    const int32_t *ho = S->hout.as<int32_t>();
    memcpy(best_idx, ho, (size_t)nq * 4);
    memcpy(best_dist, ho + nq, (size_t)nq * 4);
    memcpy(second_dist, ho + 2 * (size_t)nq, (size_t)nq * 4);
    return YGZFE_OK;
}

int ygzfe_hamming_csr(int device, const uint8_t *query, int nq, const uint8_t *train, int nt, const int32_t *row_ptr,
                      const int32_t *cand, int32_t *dist_out) {
    if (nq < 0 || nt < 0 || !row_ptr) { set_error("invalid argument"); return YGZFE_EINVAL; }
    if (nq == 0) return YGZFE_OK;
    const int nc = row_ptr[nq];
    if (nc == 0) return YGZFE_OK;
    if (!query || !train || !cand || !dist_out) { set_error("invalid argument"); return YGZFE_EINVAL; }
    for (int k = 0; k < nc; k++)
        if (cand[k] < 0 || cand[k] >= nt) { set_error("candidate index %d out of range", cand[k]); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(device));
    StagingLease S;
    YGZ_TRY(S.acquire(device));
    // in: [query][train][row_ptr][cand]  out: [dist]
    const size_t o_t = align16((size_t)nq * 32), o_r = o_t + align16((size_t)nt * 32);
    const size_t o_c = o_r + align16((size_t)(nq + 1) * 4), in_bytes = o_c + align16((size_t)nc * 4);
    const size_t out_bytes = (size_t)nc * 4;
    YGZ_TRY(S->hin.ensure(in_bytes));
    YGZ_TRY(S->hout.ensure(out_bytes));
    YGZ_TRY(S->dev.ensure(in_bytes + out_bytes));
    uint8_t *h = S->hin.as<uint8_t>(), *d = S->dev.as<uint8_t>();
    memcpy(h, query, (size_t)nq * 32);
    memcpy(h + o_t, train, (size_t)nt * 32);
    memcpy(h + o_r, row_ptr, (size_t)(nq + 1) * 4);
    memcpy(h + o_c, cand, (size_t)nc * 4);
    YGZ_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, S->stream));
    int32_t *ds = reinterpret_cast<int32_t *>(d + in_bytes);
    YGZ_HIP(launch_hamming_csr(d, nq, d + o_t, reinterpret_cast<const int32_t *>(d + o_r),
                               reinterpret_cast<const int32_t *>(d + o_c), ds, S->stream));
    YGZ_HIP(hipMemcpyAsync(S->hout.p, ds, out_bytes, hipMemcpyDeviceToHost, S->stream));
    YGZ_HIP(hipStreamSynchronize(S->stream));
    memcpy(dist_out, S->hout.p, out_bytes);
    return YGZFE_OK;
}

int ygzfe_batch_match(ygzfe_batch *b, int n_pairs, const int32_t *d_qframe, const int32_t *d_tframe,
                      int32_t *d_best_idx, int32_t *d_best_dist, int32_t *d_second_dist, void *stream) {
    if (!b || n_pairs < 0) { set_error("invalid argument"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(b->device));
    hipStream_t st = stream ? (hipStream_t)stream : b->stream;
    const Plan &P = b->plan->hp();
    hipEvent_t t0 = b->begin(st);
    YGZ_HIP(launch_hamming_best2_pairs(b->ws.desc.as<uint8_t>(), b->ws.counts.as<int32_t>(), P.kp_cap, n_pairs,
                                       d_qframe, d_tframe, d_best_idx, d_best_dist, d_second_dist, st));
    b->end(ST_HAM, t0, st);
    return YGZFE_OK;
}

// ------------------------------------------------------------------ sparse align
static AlignLevels levels_of(const Plan &P) {
    AlignLevels lv;
    memset(&lv, 0, sizeof(lv));
    for (int l = 0; l < P.nlevels; l++) {
        lv.w[l] = P.lv[l].w;
        lv.h[l] = P.lv[l].h;
        lv.off[l] = P.lv[l].off;
        lv.inv_scale[l] = P.lv[l].inv_scale;
    }
    return lv;
}

static int sparse_align_begin(const ygzfe_frame *ref, const ygzfe_frame *cur, const ygzfe_camera *cam,
                              const ygzfe_kp *kps, const float *xyz_ref, const uint8_t *usable, int n, int max_level,
                              int min_level, const ygzfe_se3 *T_init, int method) {
    if (method != YGZFE_ALIGN_GAUSS_NEWTON && method != YGZFE_ALIGN_LEVENBERG_MARQUARDT) {
        set_error("unknown SparseImgAlign method %d", method);
        return YGZFE_EINVAL;
    }
    if (!ref || !cur || !cam || !T_init || n < 0 || (n > 0 && (!kps || !xyz_ref || !usable))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (ref->plan != cur->plan) { set_error("ref and cur frames must share size and extractor"); return YGZFE_EINVAL; }
    const Plan &P = ref->plan->hp();
    if (min_level < 0 || max_level >= P.nlevels || min_level > max_level) {
        set_error("levels [%d,%d] outside the %d-level pyramid", min_level, max_level, P.nlevels);
        return YGZFE_EINVAL;
    }
    ygzfe_extractor *ex = ref->ex;
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    if (ex->align_pending) { set_error("a SparseImgAlign is already in flight on this extractor"); return YGZFE_ESTATE; }
    YGZ_TRY(ex->ensure_align_stream());
    YGZ_TRY(ex->ahout.ensure(sizeof(ygzfe_align_result)));
    if (n == 0) {  // SparseImageAlign.cc:24-27: no alignment, TCR untouched
        ygzfe_align_result *r = ex->ahout.as<ygzfe_align_result>();
        memset(r, 0, sizeof(*r));
        r->T_cur_ref = *T_init;
        r->chi2 = 1e10f;
        YGZ_HIP(hipEventRecord(ex->ev_align_done, ex->astream));
        ex->align_pending = true;
        return YGZFE_OK;
    }
    hipStream_t st = ex->astream;
    // after everything queued so far on the extractor stream (the two pyramids)
    YGZ_HIP(hipEventRecord(ex->ev_align_fork, ex->stream));
    YGZ_HIP(hipStreamWaitEvent(st, ex->ev_align_fork, 0));
    // A feature without a usable map point adds nothing to H, Jres, chi2 or the count
    // (SparseImageAlign.cc:67-75), so a reference frame with more keypoints than the
    // register kernel's threads (a keyframe after its DSO extraction, Frame.cc:717-771:
    // ~2,400 rows, only the tracked ones with map points) sends only its usable
    // features, in order, and stays on the register kernel
    const int n_all = n;
    int n_use = n;
    if (n > sparse_align_reg_capacity()) {
        n_use = 0;
        for (int i = 0; i < n; i++) n_use += usable[i] != 0;
    }
    n = n_use;
    // one packed H2D from pinned staging: [job][keypoints][xyz][usable] (16-B aligned
    // pieces), cached device buffers, one D2H of the result
    const size_t o_k = align16(sizeof(AlignJob)), o_x = o_k + align16(sizeof(ygzfe_kp) * (size_t)n);
    const size_t o_u = o_x + align16(sizeof(float) * 3 * (size_t)n), in_bytes = o_u + align16((size_t)n);
    const size_t spj = sparse_align_scratch_floats(n);
    YGZ_TRY(ex->align_in.ensure(in_bytes));
    YGZ_TRY(ex->align_scratch.ensure(sizeof(float) * spj));
    YGZ_TRY(ex->align_out.ensure(sizeof(ygzfe_align_result)));
    YGZ_TRY(ex->ahin.ensure(in_bytes));
    uint8_t *din = ex->align_in.as<uint8_t>(), *hin = ex->ahin.as<uint8_t>();
    AlignJob job;
    job.ref_pyr = ref->pyr.as<uint8_t>();
    job.cur_pyr = cur->pyr.as<uint8_t>();
    job.kps = reinterpret_cast<const ygzfe_kp *>(din + o_k);
    job.xyz = reinterpret_cast<const float *>(din + o_x);
    job.usable = din + o_u;
    job.n = n;
    job.max_level = max_level;
    job.min_level = min_level;
    job.method = method;
    job.T_init = *T_init;
    memcpy(hin, &job, sizeof(job));
    if (n == n_all) {
        memcpy(hin + o_k, kps, sizeof(ygzfe_kp) * (size_t)n);
        memcpy(hin + o_x, xyz_ref, sizeof(float) * 3 * (size_t)n);
        memcpy(hin + o_u, usable, (size_t)n);
    } else {
        ygzfe_kp *hk = reinterpret_cast<ygzfe_kp *>(hin + o_k);
        float *hx = reinterpret_cast<float *>(hin + o_x);
        for (int i = 0, j = 0; i < n_all; i++)
            if (usable[i]) {
                hk[j] = kps[i];
                memcpy(hx + 3 * (size_t)j, xyz_ref + 3 * (size_t)i, 3 * sizeof(float));
                j++;
            }
        memset(hin + o_u, 1, (size_t)n);
    }
    YGZ_HIP(hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, st));
    YGZ_HIP(launch_sparse_align(levels_of(P), *cam, reinterpret_cast<const AlignJob *>(din), 1,
                                ex->align_scratch.as<float>(), spj, ex->align_out.as<ygzfe_align_result>(), st, n,
                                method));
    YGZ_HIP(hipMemcpyAsync(ex->ahout.p, ex->align_out.p, sizeof(ygzfe_align_result), hipMemcpyDeviceToHost, st));
    YGZ_HIP(hipEventRecord(ex->ev_align_done, st));
    ex->align_pending = true;
    return YGZFE_OK;
}

int ygzfe_extractor_align_probe(ygzfe_extractor *ex, int *attempts, int *passed) {
    if (!ex) { set_error("invalid argument"); return YGZFE_EINVAL; }
    std::lock_guard<std::mutex> lk(ex->mu);
    if (attempts) *attempts = ex->align_probe_attempts;
    if (passed) *passed = ex->align_probe_beside;
    return YGZFE_OK;
}

int ygzfe_sparse_align_end(const ygzfe_frame *cur, ygzfe_align_result *result) {
    if (!cur || !result) { set_error("invalid argument"); return YGZFE_EINVAL; }
    ygzfe_extractor *ex = cur->ex;
    std::lock_guard<std::mutex> lk(ex->mu);
    if (!ex->align_pending) { set_error("no SparseImgAlign in flight on this extractor"); return YGZFE_ESTATE; }
    YGZ_TRY(ensure_device(ex->device));
    ex->align_pending = false;
    YGZ_HIP(hipEventSynchronize(ex->ev_align_done));
    memcpy(result, ex->ahout.p, sizeof(*result));
    return YGZFE_OK;
}

int ygzfe_sparse_align_begin(const ygzfe_frame *ref, const ygzfe_frame *cur, const ygzfe_camera *cam,
                             const ygzfe_kp *kps, const float *xyz_ref, const uint8_t *usable, int n, int max_level,
                             int min_level, const ygzfe_se3 *T_init) {
    return sparse_align_begin(ref, cur, cam, kps, xyz_ref, usable, n, max_level, min_level, T_init,
                              YGZFE_ALIGN_GAUSS_NEWTON);
}

int ygzfe_sparse_align(const ygzfe_frame *ref, const ygzfe_frame *cur, const ygzfe_camera *cam, const ygzfe_kp *kps,
                       const float *xyz_ref, const uint8_t *usable, int n, int max_level, int min_level,
                       const ygzfe_se3 *T_init, ygzfe_align_result *result) {
    return ygzfe_sparse_align_method(ref, cur, cam, kps, xyz_ref, usable, n, max_level, min_level, T_init,
                                     YGZFE_ALIGN_GAUSS_NEWTON, result);
}

int ygzfe_sparse_align_method(const ygzfe_frame *ref, const ygzfe_frame *cur, const ygzfe_camera *cam,
                              const ygzfe_kp *kps, const float *xyz_ref, const uint8_t *usable, int n, int max_level,
                              int min_level, const ygzfe_se3 *T_init, int method, ygzfe_align_result *result) {
    if (!result) { set_error("invalid argument"); return YGZFE_EINVAL; }
    YGZ_TRY(sparse_align_begin(ref, cur, cam, kps, xyz_ref, usable, n, max_level, min_level, T_init, method));
    return ygzfe_sparse_align_end(cur, result);
}

}  // extern "C"

namespace ygzfe {
__global__ void k_build_align_jobs(AlignJob *jobs, int n_pairs, const int32_t *ref_idx, const int32_t *cur_idx,
                                   const uint8_t *pyr, uint32_t pitch, const ygzfe_kp *kps, const int32_t *counts,
                                   int kp_cap, const float *xyz, const uint8_t *usable, int max_level, int min_level,
                                   const ygzfe_se3 *T_init) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pairs) return;
    const int r = ref_idx[p], c = cur_idx[p];
    AlignJob j;
    j.ref_pyr = pyr + (size_t)r * pitch;
    j.cur_pyr = pyr + (size_t)c * pitch;
    j.kps = kps + (size_t)r * kp_cap;
    j.xyz = xyz + (size_t)p * kp_cap * 3;
    j.usable = usable + (size_t)p * kp_cap;
    j.n = counts[r];
    j.max_level = max_level;
    j.min_level = min_level;
    j.method = 0;
    j.T_init = T_init[p];
    jobs[p] = j;
}
}  // namespace ygzfe

extern "C" int ygzfe_batch_sparse_align(ygzfe_batch *b, int n_pairs, const int32_t *d_ref_idx,
                                        const int32_t *d_cur_idx, const float *d_xyz_ref, const uint8_t *d_usable,
                                        const ygzfe_camera *cam, int max_level, int min_level,
                                        const ygzfe_se3 *d_T_init, ygzfe_align_result *d_out, void *stream) {
    if (!b || !cam || n_pairs < 0 || !d_ref_idx || !d_cur_idx || !d_xyz_ref || !d_usable || !d_T_init || !d_out) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    const Plan &P = b->plan->hp();
    if (min_level < 0 || max_level >= P.nlevels || min_level > max_level) {
        set_error("levels [%d,%d] outside the %d-level pyramid", min_level, max_level, P.nlevels);
        return YGZFE_EINVAL;
    }
    if (n_pairs == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(b->device));
    hipStream_t st = stream ? (hipStream_t)stream : b->stream;
    const size_t spj = sparse_align_scratch_floats(P.kp_cap);
    YGZ_TRY(b->jobs.ensure(sizeof(AlignJob) * n_pairs));
    YGZ_TRY(b->ascratch.ensure(sizeof(float) * spj * n_pairs));
    hipLaunchKernelGGL(k_build_align_jobs, dim3((n_pairs + 63) / 64), dim3(64), 0, st, b->jobs.as<AlignJob>(), n_pairs,
                       d_ref_idx, d_cur_idx, b->pyr.as<uint8_t>(), P.pyr_bytes, b->ws.kps.as<ygzfe_kp>(),
                       b->ws.counts.as<int32_t>(), P.kp_cap, d_xyz_ref, d_usable, max_level, min_level, d_T_init);
    YGZ_HIP(hipGetLastError());
    hipEvent_t t0 = b->begin(st);
    YGZ_HIP(launch_sparse_align(levels_of(P), *cam, b->jobs.as<AlignJob>(), n_pairs, b->ascratch.as<float>(), spj,
                                d_out, st, P.kp_cap));
    b->end(ST_ALIGN, t0, st);
    return YGZFE_OK;
}

// ------------------------------------------------------------------ Align2D / direct projection
extern "C" int ygzfe_align2d_batch(const ygzfe_frame *cur, int level, int n, const uint8_t *patches_with_border,
                                   const uint8_t *patches, int n_iter, float *px_io, uint8_t *converged) {
    if (!cur || n < 0 || (n > 0 && (!patches_with_border || !patches || !px_io || !converged))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    const Plan &P = cur->plan->hp();
    if (level < 0 || level >= P.nlevels) { set_error("level out of range"); return YGZFE_EINVAL; }
    if (n == 0) return YGZFE_OK;
    ygzfe_extractor *ex = cur->ex;
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    hipStream_t st = ex->stream;
    // in: [patches with border][patches][px]  out: [px][converged]
    const size_t o_p = align16((size_t)n * 100), o_x = o_p + align16((size_t)n * 64), in_bytes = o_x + align16((size_t)n * 8);
    const size_t out_bytes = (size_t)n * 9;
    YGZ_TRY(ex->direct_hin.ensure(in_bytes));
    YGZ_TRY(ex->direct_hout.ensure(out_bytes));
    YGZ_TRY(ex->direct_dev.ensure(in_bytes + align16(out_bytes)));
    uint8_t *h = ex->direct_hin.as<uint8_t>(), *d = ex->direct_dev.as<uint8_t>();
    memcpy(h, patches_with_border, (size_t)n * 100);
    memcpy(h + o_p, patches, (size_t)n * 64);
    memcpy(h + o_x, px_io, (size_t)n * 8);
    YGZ_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, st));
    float *dpx = reinterpret_cast<float *>(d + in_bytes);
    uint8_t *dconv = d + in_bytes + (size_t)n * 8;
    YGZ_HIP(hipMemcpyAsync(dpx, d + o_x, (size_t)n * 8, hipMemcpyDeviceToDevice, st));
    const LevelDesc &L = P.lv[level];
    YGZ_HIP(launch_align2d(cur->pyr.as<uint8_t>() + L.off, L.w, L.h, n, d, d + o_p, n_iter, dpx, dconv, st));
    YGZ_HIP(hipMemcpyAsync(ex->direct_hout.p, dpx, out_bytes, hipMemcpyDeviceToHost, st));
    YGZ_HIP(hipStreamSynchronize(st));
    memcpy(px_io, ex->direct_hout.p, (size_t)n * 8);
    memcpy(converged, ex->direct_hout.as<uint8_t>() + (size_t)n * 8, (size_t)n);
    return YGZFE_OK;
}

// FAST-10 (Thirdparty/fast) over host-image ROIs: the whole image and the ROI table
// go up in one DMA, one workgroup per ROI, the corner lists come back in one.
extern "C" int ygzfe_fast10_detect(int device, const uint8_t *img, int width, int height, int stride,
                                   const int32_t *rois, int n_roi, int barrier, int variant, int16_t *xy, int cap,
                                   int32_t *counts) {
    if (!img || width <= 0 || height <= 0 || stride < width || n_roi < 0 || (n_roi > 0 && (!rois || !counts)) ||
        cap < 0 || (cap > 0 && !xy) || (variant != 0 && variant != 1) || barrier < 0) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    for (int r = 0; r < n_roi; r++) {
        const int x0 = rois[4 * r], y0 = rois[4 * r + 1], w = rois[4 * r + 2], h = rois[4 * r + 3];
        if (w < 0 || h < 0) { set_error("roi %d: negative size", r); return YGZFE_EINVAL; }
        // the tested pixels (the whole ROI for the plain scan, its [3, -3) interior for SSE2
        // when w >= 22) with their radius-3 rings
        const int in = (variant == 1 && w >= 22) ? 3 : 0;
        if (w - 2 * in <= 0 || h - 2 * in <= 0) continue;
        if (x0 + in - 3 < 0 || y0 + in - 3 < 0 || x0 + w - in + 3 > width || y0 + h - in + 3 > height) {
            set_error("roi %d (%d, %d, %d, %d): the segment test would read outside the %dx%d image", r, x0, y0, w,
                      h, width, height);
            return YGZFE_EINVAL;
        }
    }
    if (n_roi == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(device));
    StagingLease S;
    YGZ_TRY(S.acquire(device));
    // in: [image][rois]  out: [counts][xy]
    const size_t img_b = (size_t)stride * height, o_r = align16(img_b), in_bytes = o_r + align16((size_t)n_roi * 16);
    const size_t o_xy = align16((size_t)n_roi * 4), out_bytes = o_xy + (size_t)n_roi * cap * 4;
    YGZ_TRY(S->hin.ensure(in_bytes));
    YGZ_TRY(S->hout.ensure(out_bytes));
    YGZ_TRY(S->dev.ensure(in_bytes + out_bytes));
    uint8_t *h = S->hin.as<uint8_t>(), *d = S->dev.as<uint8_t>();
    // the caller's last row may hold only `width` bytes (a cv::Mat ROI view)
    memcpy(h, img, (size_t)(height - 1) * stride + width);
    memcpy(h + o_r, rois, (size_t)n_roi * 16);
    YGZ_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, S->stream));
    int32_t *dc = reinterpret_cast<int32_t *>(d + in_bytes);
    int16_t *dxy = reinterpret_cast<int16_t *>(d + in_bytes + o_xy);
    YGZ_HIP(launch_fast10_rois(d, stride, reinterpret_cast<const int *>(d + o_r), n_roi, barrier, variant, dxy, cap,
                               dc, S->stream));
    YGZ_HIP(hipMemcpyAsync(S->hout.p, dc, out_bytes, hipMemcpyDeviceToHost, S->stream));
    YGZ_HIP(hipStreamSynchronize(S->stream));
    memcpy(counts, S->hout.p, (size_t)n_roi * 4);
    if (cap > 0) memcpy(xy, S->hout.as<uint8_t>() + o_xy, (size_t)n_roi * cap * 4);
    for (int r = 0; r < n_roi; r++)
        if (counts[r] > cap) {
            set_error("roi %d: %d corners > cap %d", r, counts[r], cap);
            return YGZFE_ECAP;
        }
    return YGZFE_OK;
}

extern "C" int ygzfe_debug_dso_cells(int device, const uint8_t *img, int width, int height, int g, int barrier,
                                     uint8_t *flags) {
    if (!img || !flags || width <= 0 || height <= 0 || g < 7 || g > kDsoMaxGridHost) {
        set_error("invalid argument (g in [7, %d])", kDsoMaxGridHost);
        return YGZFE_EINVAL;
    }
    const size_t ncells = (size_t)(height / g) * (width / g), img_b = (size_t)width * height;
    const size_t o_f = align16(img_b), fb = ncells * g * g;
    if (ncells == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(device));
    StagingLease S;
    YGZ_TRY(S.acquire(device));
    YGZ_TRY(S->hin.ensure(img_b));
    YGZ_TRY(S->hout.ensure(fb));
    YGZ_TRY(S->dev.ensure(o_f + fb));
    uint8_t *d = S->dev.as<uint8_t>();
    memcpy(S->hin.p, img, img_b);
    YGZ_HIP(hipMemcpyAsync(d, S->hin.p, img_b, hipMemcpyHostToDevice, S->stream));
    YGZ_HIP(launch_dso_cells_debug(d, width, height, g, barrier, d + o_f, S->stream));
    YGZ_HIP(hipMemcpyAsync(S->hout.p, d + o_f, fb, hipMemcpyDeviceToHost, S->stream));
    YGZ_HIP(hipStreamSynchronize(S->stream));
    memcpy(flags, S->hout.p, fb);
    return YGZFE_OK;
}

// Align2D(const cv::Mat& cur_img, ...) on a host image: the 48 x 48 window around
// the estimate goes up (the whole image only when the iterations walk out of it).
extern "C" int ygzfe_align2d_image(int device, const uint8_t *img, int w, int h, int stride,
                                   const uint8_t *patch_with_border, const uint8_t *patch, int n_iter, float *px,
                                   uint8_t *converged) {
    if (!img || w <= 0 || h <= 0 || stride < w || !patch_with_border || !patch || !px || !converged) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    YGZ_TRY(ensure_device(device));
    StagingLease S;
    YGZ_TRY(S.acquire(device));
    hipStream_t st = S->stream;
    const size_t small = 256;  // pwb 100 | p 64 | px 8 | status 4
    uint8_t host_small[small];
    memcpy(host_small, patch_with_border, 100);
    memcpy(host_small + 100, patch, 64);
    memcpy(host_small + 164, px, 8);
    const int half = 24;
    float fu = px[0], fv = px[1];
    int cu = std::isfinite(fu) ? (int)floorf(fu) : 0, cv = std::isfinite(fv) ? (int)floorf(fv) : 0;
    cu = std::min(std::max(cu, 0), w - 1);
    cv = std::min(std::max(cv, 0), h - 1);
    for (int pass = 0; pass < 2; pass++) {
        int x0 = 0, y0 = 0, ww = w, wh = h;
        if (pass == 0) {
            x0 = std::max(cu - half, 0);
            y0 = std::max(cv - half, 0);
            ww = std::min(cu + half, w) - x0;
            wh = std::min(cv + half, h) - y0;
        }
        YGZ_TRY(S->dev.ensure(small + (size_t)ww * wh));
        uint8_t *d = S->dev.as<uint8_t>();
        YGZ_HIP(hipMemcpyAsync(d, host_small, 172, hipMemcpyHostToDevice, st));
        YGZ_HIP(hipMemcpy2DAsync(d + small, ww, img + (size_t)y0 * stride + x0, stride, ww, wh,
                                 hipMemcpyHostToDevice, st));
        YGZ_HIP(launch_align2d_window(d + small, ww, w, h, x0, y0, ww, wh, d, d + 100, n_iter,
                                      reinterpret_cast<float *>(d + 164), reinterpret_cast<int *>(d + 172), st));
        uint8_t back[12];
        YGZ_HIP(hipMemcpyAsync(back, d + 164, 12, hipMemcpyDeviceToHost, st));
        YGZ_HIP(hipStreamSynchronize(st));
        int status;
        memcpy(&status, back + 8, 4);
        if (status >= 0) {
            memcpy(px, back, 8);
            *converged = (uint8_t)status;
            return YGZFE_OK;
        }
    }
    set_error("Align2D window retry failed");
    return YGZFE_EHIP;
}

extern "C" int ygzfe_find_direct_projection_batch(const ygzfe_frame *const *ref, const ygzfe_frame *cur,
                                                  const ygzfe_camera *cam, int n, const int32_t *ref_index,
                                                  const ygzfe_kp *kp_ref, const float *pt_ref, const ygzfe_se3 *T_cr,
                                                  float *px_io, int32_t *search_level, uint8_t *ok) {
    if (!ref || !cur || !cam || n < 0 ||
        (n > 0 && (!ref_index || !kp_ref || !pt_ref || !T_cr || !px_io || !search_level || !ok))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (n == 0) return YGZFE_OK;
    int nref = 0;
    for (int i = 0; i < n; i++) nref = std::max(nref, ref_index[i] + 1);
    for (int i = 0; i < n; i++)
        if (ref_index[i] < 0) { set_error("negative ref_index"); return YGZFE_EINVAL; }
    for (int r = 0; r < nref; r++)
        if (!ref[r] || ref[r]->plan != cur->plan) {
            set_error("reference keyframe %d missing or of a different size", r);
            return YGZFE_EINVAL;
        }
    ygzfe_extractor *ex = cur->ex;
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    hipStream_t st = ex->stream;
    const Plan &P = cur->plan->hp();
    // in: [ref ptrs][scale][ref_index][kps][pt][T]  out: [px][level][ok]
    const size_t o_sc = align16(sizeof(void *) * nref), o_ri = o_sc + align16(sizeof(float) * P.nlevels);
    const size_t o_kp = o_ri + align16(4 * (size_t)n), o_pt = o_kp + align16(sizeof(ygzfe_kp) * n);
    const size_t o_T = o_pt + align16(12 * (size_t)n), o_px = o_T + align16(sizeof(ygzfe_se3) * n);
    const size_t in_bytes = o_px + align16(8 * (size_t)n), out_bytes = (size_t)n * 13;
    YGZ_TRY(ex->direct_hin.ensure(in_bytes));
    YGZ_TRY(ex->direct_hout.ensure(out_bytes));
    YGZ_TRY(ex->direct_dev.ensure(in_bytes + align16(out_bytes)));
    uint8_t *h = ex->direct_hin.as<uint8_t>(), *d = ex->direct_dev.as<uint8_t>();
    const uint8_t **ptrs = reinterpret_cast<const uint8_t **>(h);
    for (int r = 0; r < nref; r++) ptrs[r] = ref[r]->pyr.as<uint8_t>();
    float *sc = reinterpret_cast<float *>(h + o_sc);
    for (int l = 0; l < P.nlevels; l++) sc[l] = P.lv[l].scale;
    memcpy(h + o_ri, ref_index, 4 * (size_t)n);
    memcpy(h + o_kp, kp_ref, sizeof(ygzfe_kp) * n);
    memcpy(h + o_pt, pt_ref, 12 * (size_t)n);
    memcpy(h + o_T, T_cr, sizeof(ygzfe_se3) * n);
    memcpy(h + o_px, px_io, 8 * (size_t)n);
    YGZ_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, st));
    float *dpx = reinterpret_cast<float *>(d + in_bytes);
    int32_t *dlv = reinterpret_cast<int32_t *>(d + in_bytes + 8 * (size_t)n);
    uint8_t *dok = d + in_bytes + 12 * (size_t)n;
    YGZ_HIP(hipMemcpyAsync(dpx, d + o_px, 8 * (size_t)n, hipMemcpyDeviceToDevice, st));
    const AlignLevels lv = levels_of(P);
    YGZ_HIP(launch_find_direct(reinterpret_cast<const uint8_t *const *>(d), lv, cur->pyr.as<uint8_t>(), lv, P.nlevels,
                               reinterpret_cast<const float *>(d + o_sc), ex->scales.inv_sigma2[1 < P.nlevels ? 1 : 0],
                               *cam, n, reinterpret_cast<const int32_t *>(d + o_ri),
                               reinterpret_cast<const ygzfe_kp *>(d + o_kp), reinterpret_cast<const float *>(d + o_pt),
                               reinterpret_cast<const ygzfe_se3 *>(d + o_T), dpx, dlv, dok, st));
    YGZ_HIP(hipMemcpyAsync(ex->direct_hout.p, dpx, out_bytes, hipMemcpyDeviceToHost, st));
    YGZ_HIP(hipStreamSynchronize(st));
    const uint8_t *ho = ex->direct_hout.as<uint8_t>();
    memcpy(px_io, ho, 8 * (size_t)n);
    memcpy(search_level, ho + 8 * (size_t)n, 4 * (size_t)n);
    memcpy(ok, ho + 12 * (size_t)n, (size_t)n);
    return YGZFE_OK;
}

// SearchLocalPointsDirect (Tracking.cc:2258-2410): items of both phases in one
// packed H2D from pinned staging, k_direct_items + k_direct_replay, one packed D2H.
static int search_direct_impl(const ygzfe_frame *const *ref, int n_ref, const ygzfe_frame *cur,
                              const ygzfe_camera *cam, int n_cache, int n_local, const int32_t *item_ptr,
                              const int32_t *ref_index, const ygzfe_kp *kp_ref, const float *pt_ref,
                              const ygzfe_se3 *T_cr, const float *px_proj, float border, int grid_size,
                              int cache_hit_th, float *px_out, int32_t *matched_item, int32_t *status,
                              int *cache_success, int *local_ran) {
    const int n_points = n_cache + n_local;
    if (!ref || n_ref < 0 || !cur || !cam || n_cache < 0 || n_local < 0 ||
        (n_points > 0 && (!item_ptr || !px_proj || !px_out || !matched_item))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (grid_size <= 0) { set_error("grid_size must be positive"); return YGZFE_EINVAL; }
    const Plan &P = cur->plan->hp();
    const long ncell = (long)(P.lv[0].h / grid_size) * (P.lv[0].w / grid_size);
    if (ncell > kDirectMaxGridCells) {
        set_error("coverage grid of %ld cells exceeds %d", ncell, kDirectMaxGridCells);
        return YGZFE_EINVAL;
    }
    if (n_points == 0) {
        if (cache_success) *cache_success = 0;
        if (local_ran) *local_ran = !(0 > cache_hit_th);
        return YGZFE_OK;
    }
    if (item_ptr[0] != 0) { set_error("item_ptr[0] must be 0"); return YGZFE_EINVAL; }
    for (int i = 0; i < n_points; i++)
        if (item_ptr[i + 1] < item_ptr[i]) { set_error("item_ptr not monotone at %d", i); return YGZFE_EINVAL; }
    const int n_items = item_ptr[n_points];
    if (n_items > 0 && (!ref_index || !kp_ref || !pt_ref || !T_cr)) { set_error("null item array"); return YGZFE_EINVAL; }
    for (int k = 0; k < n_items; k++)
        if (ref_index[k] < 0 || ref_index[k] >= n_ref) { set_error("ref_index[%d] out of range", k); return YGZFE_EINVAL; }
    for (int k = 0; k < n_items; k++)
        if (kp_ref[k].octave < 0 || kp_ref[k].octave >= P.nlevels) {
            set_error("kp_ref[%d].octave %d out of range", k, kp_ref[k].octave);
            return YGZFE_EINVAL;
        }
    for (int r = 0; r < n_ref; r++)
        if (!ref[r] || ref[r]->plan != cur->plan) {
            set_error("reference keyframe %d missing or of a different size", r);
            return YGZFE_EINVAL;
        }
    ygzfe_extractor *ex = cur->ex;
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    hipStream_t st = ex->stream;
    // in: [ref ptrs][scale][item_ptr][px_proj][items][T table]   out: [hdr][px_out][matched][status] | [px_item][ok_item]
    // T table: one T_cr per keyframe slot while its items agree (Tracking's TCR is per
    // keyframe), else one per differing item
    std::vector<int32_t> slot_tcr((size_t)std::max(1, n_ref), -1);
    std::vector<ygzfe_se3> tab;
    tab.reserve(std::max(1, n_ref));
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_ptr = 0, o_sc = al(o_ptr + sizeof(void *) * std::max(1, n_ref));
    const size_t o_ip = al(o_sc + 4 * kMaxLevels), o_pp = al(o_ip + 4 * ((size_t)n_points + 1));
    const size_t o_it = al(o_pp + 8 * (size_t)n_points), o_tab = al(o_it + sizeof(DirectItem) * (size_t)n_items);
    std::vector<int32_t> tcr_of((size_t)n_items);
    for (int k = 0; k < n_items; k++) {
        int &e = slot_tcr[ref_index[k]];
        if (e < 0 || memcmp(&tab[e], &T_cr[k], sizeof(ygzfe_se3)) != 0) {
            const int t = (int)tab.size();
            tab.push_back(T_cr[k]);
            if (e < 0) e = t;
            tcr_of[k] = t;
        } else {
            tcr_of[k] = e;
        }
    }
    const size_t in_bytes = al(o_tab + sizeof(ygzfe_se3) * std::max<size_t>(1, tab.size()));
    const size_t o_hdr = 0, o_pxo = 16, o_m = o_pxo + 8 * (size_t)n_points, o_st = o_m + 4 * (size_t)n_points;
    const size_t back_bytes = o_st + 4 * (size_t)n_points;
    const size_t o_pxi = al(back_bytes), o_ok = al(o_pxi + 8 * (size_t)n_items), out_bytes = al(o_ok + (size_t)n_items);
    YGZ_TRY(ex->direct_hin.ensure(in_bytes));
    YGZ_TRY(ex->direct_hout.ensure(back_bytes));
    uint8_t *h = ex->direct_hin.as<uint8_t>();
    const uint8_t **ptrs = (const uint8_t **)(h + o_ptr);
    for (int r = 0; r < n_ref; r++) ptrs[r] = ref[r]->pyr.as<uint8_t>();
    float *sc = (float *)(h + o_sc);
    for (int l = 0; l < P.nlevels; l++) sc[l] = P.lv[l].scale;
    memcpy(h + o_ip, item_ptr, 4 * ((size_t)n_points + 1));
    memcpy(h + o_pp, px_proj, 8 * (size_t)n_points);
    DirectItem *it = (DirectItem *)(h + o_it);
    for (int i = 0; i < n_points; i++)
        for (int k = item_ptr[i]; k < item_ptr[i + 1]; k++) {
            it[k].kp = kp_ref[k];
            memcpy(it[k].pt, pt_ref + 3 * (size_t)k, 12);
            it[k].ref = ref_index[k];
            it[k].point = i;
            it[k].tcr = tcr_of[k];
        }
    if (!tab.empty()) memcpy(h + o_tab, tab.data(), sizeof(ygzfe_se3) * tab.size());
    YGZ_TRY(ex->direct_dev.ensure(in_bytes + out_bytes));
    uint8_t *d = ex->direct_dev.as<uint8_t>(), *dout = d + in_bytes;
    YGZ_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, st));
    YGZ_HIP(launch_search_direct((const uint8_t *const *)(d + o_ptr), levels_of(P), cur->pyr.as<uint8_t>(),
                                 P.nlevels, (const float *)(d + o_sc), ex->scales.inv_sigma2[1 < P.nlevels ? 1 : 0],
                                 *cam, n_cache, n_local, n_items, (const int32_t *)(d + o_ip), d + o_it,
                                 (const ygzfe_se3 *)(d + o_tab), (const float *)(d + o_pp), (float *)(dout + o_pxi), dout + o_ok, border, grid_size,
                                 cache_hit_th, (float *)(dout + o_pxo), (int32_t *)(dout + o_m),
                                 (int32_t *)(dout + o_st), (int32_t *)(dout + o_hdr), st));
    uint8_t *hb = ex->direct_hout.as<uint8_t>();
    YGZ_HIP(hipMemcpyAsync(hb, dout, back_bytes, hipMemcpyDeviceToHost, st));
    YGZ_HIP(hipStreamSynchronize(st));
    memcpy(px_out, hb + o_pxo, 8 * (size_t)n_points);
    memcpy(matched_item, hb + o_m, 4 * (size_t)n_points);
    if (status) memcpy(status, hb + o_st, 4 * (size_t)n_points);
    int32_t hdr[2];
    memcpy(hdr, hb + o_hdr, 8);
    if (cache_success) *cache_success = hdr[0];
    if (local_ran) *local_ran = hdr[1];
    return YGZFE_OK;
}

extern "C" int ygzfe_search_direct_batch(const ygzfe_frame *const *ref, int n_ref, const ygzfe_frame *cur,
                                         const ygzfe_camera *cam, int n_points, const int32_t *item_ptr,
                                         const int32_t *ref_index, const ygzfe_kp *kp_ref, const float *pt_ref,
                                         const ygzfe_se3 *T_cr, const float *px_proj, float border,
                                         float *px_out, int32_t *matched_item) {
    // the local-map loop alone (Tracking.cc:2348-2405): no grid, always runs
    return search_direct_impl(ref, n_ref, cur, cam, 0, n_points, item_ptr, ref_index, kp_ref, pt_ref, T_cr, px_proj,
                              border, 5, 0x7fffffff, px_out, matched_item, nullptr, nullptr, nullptr);
}

extern "C" int ygzfe_search_local_points_direct(const ygzfe_frame *const *ref, int n_ref, const ygzfe_frame *cur,
                                                const ygzfe_camera *cam, int n_cache, int n_local,
                                                const int32_t *item_ptr, const int32_t *ref_index,
                                                const ygzfe_kp *kp_ref, const float *pt_ref, const ygzfe_se3 *T_cr,
                                                const float *px_proj, float border, int grid_size, int cache_hit_th,
                                                float *px_out, int32_t *matched_item, int32_t *status,
                                                int *cache_success, int *local_ran) {
    return search_direct_impl(ref, n_ref, cur, cam, n_cache, n_local, item_ptr, ref_index, kp_ref, pt_ref, T_cr,
                              px_proj, border, grid_size, cache_hit_th, px_out, matched_item, status, cache_success,
                              local_ran);
}

// --------------------------------------------------------------------------
// Stereo (Frame.cc:509-700)
static StereoLevels stereo_levels_of(const Plan &P) {
    StereoLevels lv;
    memset(&lv, 0, sizeof(lv));
    for (int l = 0; l < P.nlevels; l++) {
        lv.w[l] = P.lv[l].w;
        lv.h[l] = P.lv[l].h;
        lv.off[l] = P.lv[l].off;
        lv.scale[l] = P.lv[l].scale;
        lv.inv_scale[l] = P.lv[l].inv_scale;
    }
    return lv;
}

static bool same_layout(const Plan &a, const Plan &b) {
    if (a.nlevels != b.nlevels) return false;
    for (int l = 0; l < a.nlevels; l++)
        if (a.lv[l].w != b.lv[l].w || a.lv[l].h != b.lv[l].h || a.lv[l].off != b.lv[l].off ||
            a.lv[l].scale != b.lv[l].scale)
            return false;
    return true;
}

static int check_octaves(const ygzfe_kp *k, int n, int nlevels) {
    for (int i = 0; i < n; i++)
        if (k[i].octave < 0 || k[i].octave >= nlevels) {
            set_error("keypoint %d octave %d outside [0, %d)", i, k[i].octave, nlevels);
            return YGZFE_EINVAL;
        }
    return YGZFE_OK;
}

extern "C" int ygzfe_stereo_matches(const ygzfe_frame *left, const ygzfe_frame *right, const ygzfe_kp *kl,
                                    const uint8_t *dl, int nl, const ygzfe_kp *kr, const uint8_t *dr, int nr,
                                    float mb, float mbf, float *u_right, float *depth) {
    if (!left || !right || nl < 0 || nr < 0 || (nl > 0 && (!kl || !dl || !u_right || !depth)) ||
        (nr > 0 && (!kr || !dr))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (!same_layout(left->plan->hp(), right->plan->hp())) {
        set_error("left and right pyramids differ in level sizes");
        return YGZFE_EINVAL;
    }
    if (nr > 65535) { set_error("more than 65535 right keypoints"); return YGZFE_EINVAL; }
    if (!(mb > 0.f)) { set_error("baseline must be positive"); return YGZFE_EINVAL; }
    if (nl == 0) return YGZFE_OK;
    const Plan &P = left->plan->hp();
    YGZ_TRY(check_octaves(kl, nl, P.nlevels));
    YGZ_TRY(check_octaves(kr, nr, P.nlevels));
    ygzfe_extractor *ex = left->ex;
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    hipStream_t st = ex->stream;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    // in: [job][counts][kl][kr][dl][dr]  out: [u_right][depth][sad]
    const size_t o_job = 0, o_cnt = al(sizeof(StereoJob)), o_kl = al(o_cnt + 8);
    const size_t o_kr = al(o_kl + sizeof(ygzfe_kp) * (size_t)nl), o_dl = al(o_kr + sizeof(ygzfe_kp) * (size_t)nr);
    const size_t o_dr = al(o_dl + 32 * (size_t)nl), in_bytes = al(o_dr + 32 * (size_t)nr);
    const size_t o_u = in_bytes, o_d = al(o_u + 4 * (size_t)nl), o_s = al(o_d + 4 * (size_t)nl);
    const size_t total = al(o_s + 4 * (size_t)nl);
    YGZ_TRY(ex->direct_dev.ensure(total));
    uint8_t *d = ex->direct_dev.as<uint8_t>();
    YGZ_TRY(ex->direct_hin.ensure(in_bytes));
    uint8_t *h = ex->direct_hin.as<uint8_t>();
    StereoJob J;
    J.left_pyr = left->pyr.as<uint8_t>();
    J.right_pyr = right->pyr.as<uint8_t>();
    J.left_kps = (const ygzfe_kp *)(d + o_kl);
    J.right_kps = (const ygzfe_kp *)(d + o_kr);
    J.left_desc = d + o_dl;
    J.right_desc = d + o_dr;
    J.n_left = (const int *)(d + o_cnt);
    J.n_right = (const int *)(d + o_cnt + 4);
    J.u_right = (float *)(d + o_u);
    J.depth = (float *)(d + o_d);
    J.sad = (int *)(d + o_s);
    memcpy(h + o_job, &J, sizeof(J));
    const int cnt[2] = {nl, nr};
    memcpy(h + o_cnt, cnt, 8);
    memcpy(h + o_kl, kl, sizeof(ygzfe_kp) * (size_t)nl);
    if (nr) memcpy(h + o_kr, kr, sizeof(ygzfe_kp) * (size_t)nr);
    memcpy(h + o_dl, dl, 32 * (size_t)nl);
    if (nr) memcpy(h + o_dr, dr, 32 * (size_t)nr);
    YGZ_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, st));
    YGZ_HIP(launch_stereo((const StereoJob *)(d + o_job), 1, nl, stereo_levels_of(P), mb, mbf, st));
    YGZ_HIP(hipMemcpyAsync(u_right, d + o_u, 4 * (size_t)nl, hipMemcpyDeviceToHost, st));
    YGZ_HIP(hipMemcpyAsync(depth, d + o_d, 4 * (size_t)nl, hipMemcpyDeviceToHost, st));
    YGZ_HIP(hipStreamSynchronize(st));
    return YGZFE_OK;
}

extern "C" int ygzfe_batch_stereo(ygzfe_batch *b, int n_pairs, const int32_t *d_left_idx, const int32_t *d_right_idx,
                                  float mb, float mbf, float *d_u_right, float *d_depth, void *stream) {
    if (!b || n_pairs < 0 || (n_pairs > 0 && (!d_left_idx || !d_right_idx || !d_u_right || !d_depth))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (!(mb > 0.f)) { set_error("baseline must be positive"); return YGZFE_EINVAL; }
    if (n_pairs == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(b->device));
    hipStream_t st = stream ? (hipStream_t)stream : b->stream;
    const Plan &P = b->plan->hp();
    if (P.kp_cap > 65535) { set_error("kp_cap exceeds 65535"); return YGZFE_EINVAL; }
    YGZ_TRY(b->sjobs.ensure(sizeof(StereoJob) * (size_t)n_pairs));
    YGZ_TRY(b->ssad.ensure(4 * (size_t)n_pairs * P.kp_cap));
    hipEvent_t t0 = b->begin(st);
    YGZ_HIP(launch_build_stereo_jobs(n_pairs, b->pyr.as<uint8_t>(), P.pyr_bytes, b->ws.kps.as<ygzfe_kp>(),
                                     b->ws.desc.as<uint8_t>(), b->ws.counts.as<int>(), P.kp_cap, d_left_idx,
                                     d_right_idx, d_u_right, d_depth, b->ssad.as<int>(), b->sjobs.as<StereoJob>(),
                                     st));
    YGZ_HIP(launch_stereo(b->sjobs.as<StereoJob>(), n_pairs, P.kp_cap, stereo_levels_of(P), mb, mbf, st));
    b->end(ST_STEREO, t0, st);
    return YGZFE_OK;
}

extern "C" int ygzfe_stereo_from_rgbd(int device, const float *im_depth, int width, int height, int stride,
                                      const ygzfe_kp *kps, int n, float mbf, float *u_right, float *depth) {
    if (!im_depth || width <= 0 || height <= 0 || stride < width || n < 0 ||
        (n > 0 && (!kps || !u_right || !depth))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (n == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(device));
    StagingLease S;
    YGZ_TRY(S.acquire(device));
    // in: [depth image][kps]  out: [u_right][depth]
    const size_t img = 4 * (size_t)stride * height, o_k = align16(img);
    const size_t in_bytes = o_k + align16(sizeof(ygzfe_kp) * (size_t)n), out_bytes = 8 * (size_t)n;
    YGZ_TRY(S->hin.ensure(in_bytes));
    YGZ_TRY(S->hout.ensure(out_bytes));
    YGZ_TRY(S->dev.ensure(in_bytes + out_bytes));
    uint8_t *h = S->hin.as<uint8_t>(), *d = S->dev.as<uint8_t>();
    memcpy(h, im_depth, 4 * ((size_t)(height - 1) * stride + width));  // the last row may end at `width`
    memcpy(h + o_k, kps, sizeof(ygzfe_kp) * (size_t)n);
    YGZ_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, S->stream));
    float *du = reinterpret_cast<float *>(d + in_bytes), *dd = du + n;
    YGZ_HIP(launch_stereo_rgbd(reinterpret_cast<const float *>(d), 0, width, height, stride,
                               reinterpret_cast<const ygzfe_kp *>(d + o_k), n, nullptr, n, 1, mbf, du, dd, S->stream));
    YGZ_HIP(hipMemcpyAsync(S->hout.p, du, out_bytes, hipMemcpyDeviceToHost, S->stream));
    YGZ_HIP(hipStreamSynchronize(S->stream));
    memcpy(u_right, S->hout.p, 4 * (size_t)n);
    memcpy(depth, S->hout.as<float>() + n, 4 * (size_t)n);
    return YGZFE_OK;
}

extern "C" int ygzfe_batch_stereo_rgbd(ygzfe_batch *b, int n_frames, const float *d_depth_images,
                                       size_t depth_pitch, int stride, float mbf, float *d_u_right, float *d_depth,
                                       void *stream) {
    if (!b || n_frames < 0 || (n_frames > 0 && (!d_depth_images || !d_u_right || !d_depth))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (n_frames > b->maxF) { set_error("n_frames %d > batch capacity %d", n_frames, b->maxF); return YGZFE_EINVAL; }
    if (n_frames == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(b->device));
    hipStream_t st = stream ? (hipStream_t)stream : b->stream;
    const Plan &P = b->plan->hp();
    if (stride < P.lv[0].w) { set_error("depth stride < width"); return YGZFE_EINVAL; }
    YGZ_HIP(launch_stereo_rgbd(d_depth_images, depth_pitch, P.lv[0].w, P.lv[0].h, stride, b->ws.kps.as<ygzfe_kp>(),
                               P.kp_cap, b->ws.counts.as<int>(), P.kp_cap, n_frames, mbf, d_u_right, d_depth, st));
    return YGZFE_OK;
}

// --------------------------------------------------------------------------
// DBoW2 vocabulary + Frame::ComputeBoW (Frame.cc:495-500)
struct ygzfe_vocab {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0, n_nodes = 0, n_words = 0;
    DevBuf child_ptr, slot_node, slot_desc, word_id, weight;
    DevBuf scratch;
    HostBuf hin, hout;  // pinned staging of the single-frame calls (one DMA each way)
    hipStream_t stream = nullptr;
    std::mutex mu;
    VocabDev dev() const {
        VocabDev V;
        V.n_nodes = n_nodes;
        V.L = L;
        V.child_ptr = child_ptr.as<int32_t>();
        V.slot_node = slot_node.as<int32_t>();
        V.slot_desc = slot_desc.as<uint8_t>();
        V.word_id = word_id.as<int32_t>();
        V.weight = weight.as<double>();
        return V;
    }
};

// nodes as TemplatedVocabulary::loadFromTextFile leaves them (TemplatedVocabulary.h:1362-1448)
static int vocab_build(int device, int k, int L, int scoring, int weighting, int n, const int32_t *parent,
                       const uint8_t *is_leaf, const uint8_t *desc, const double *weight, ygzfe_vocab **out) {
    if (!out || n < 1 || (n > 1 && (!parent || !is_leaf || !desc || !weight))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3) {
        set_error("vocabulary header k=%d L=%d scoring=%d weighting=%d outside DBoW2's accepted ranges", k, L, scoring,
                  weighting);
        return YGZFE_EINVAL;
    }
    std::vector<int32_t> cptr((size_t)n + 1, 0), slot_node((size_t)std::max(1, n - 1)), wid((size_t)n, 0);
    std::vector<uint8_t> sdesc((size_t)std::max(1, n - 1) * 32);
    std::vector<double> w((size_t)n, 0.0);
    for (int i = 1; i < n; i++) {
        if (parent[i] < 0 || parent[i] >= i) {
            set_error("node %d: parent %d is not an earlier node", i, parent[i]);
            return YGZFE_EINVAL;
        }
        cptr[parent[i] + 1]++;
    }
    for (int i = 0; i < n; i++) {
        if (cptr[i + 1] > 255) { set_error("node %d has %d > 255 children", i, cptr[i + 1]); return YGZFE_EINVAL; }
        cptr[i + 1] += cptr[i];
    }
    std::vector<int32_t> fill(cptr.begin(), cptr.end() - 1);
    int words = 0;
    for (int i = 1; i < n; i++) {
        const int sl = fill[parent[i]]++;  // children.push_back in node order
        slot_node[sl] = i;
        memcpy(&sdesc[(size_t)sl * 32], desc + (size_t)i * 32, 32);
        w[i] = weight[i];
        if (is_leaf[i]) wid[i] = words++;
    }
    YGZ_TRY(ensure_device(device));
    std::unique_ptr<ygzfe_vocab> v(new ygzfe_vocab());
    v->device = device;
    v->k = k;
    v->L = L;
    v->scoring = scoring;
    v->weighting = weighting;
    v->n_nodes = n;
    v->n_words = words;
    YGZ_TRY(v->child_ptr.ensure(4 * cptr.size()));
    YGZ_TRY(v->slot_node.ensure(4 * slot_node.size()));
    YGZ_TRY(v->slot_desc.ensure(sdesc.size()));
    YGZ_TRY(v->word_id.ensure(4 * wid.size()));
    YGZ_TRY(v->weight.ensure(8 * w.size()));
    YGZ_HIP(hipMemcpy(v->child_ptr.p, cptr.data(), 4 * cptr.size(), hipMemcpyHostToDevice));
    YGZ_HIP(hipMemcpy(v->slot_node.p, slot_node.data(), 4 * slot_node.size(), hipMemcpyHostToDevice));
    YGZ_HIP(hipMemcpy(v->slot_desc.p, sdesc.data(), sdesc.size(), hipMemcpyHostToDevice));
    YGZ_HIP(hipMemcpy(v->word_id.p, wid.data(), 4 * wid.size(), hipMemcpyHostToDevice));
    YGZ_HIP(hipMemcpy(v->weight.p, w.data(), 8 * w.size(), hipMemcpyHostToDevice));
    YGZ_HIP(hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking));
    *out = v.release();
    return YGZFE_OK;
}

extern "C" int ygzfe_vocab_create(int device, int k, int L, int scoring, int weighting, int n_nodes,
                                  const int32_t *parent, const uint8_t *is_leaf, const uint8_t *desc,
                                  const double *weight, ygzfe_vocab **out) {
    return vocab_build(device, k, L, scoring, weighting, n_nodes, parent, is_leaf, desc, weight, out);
}

extern "C" int ygzfe_vocab_load_text(int device, const char *path, ygzfe_vocab **out) {
    // TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1362-1448), e.g. Vocabulary/ORBvoc.txt.
    // Lines holding only whitespace are skipped (the reference turns a trailing
    // empty line into an uninitialised child of the root).
    if (!path || !out) { set_error("invalid argument"); return YGZFE_EINVAL; }
    FILE *fp = fopen(path, "r");
    if (!fp) { set_error("cannot open %s", path); return YGZFE_EINVAL; }
    int k = -1, L = -1, n1 = -1, n2 = -1;
    std::string line;
    auto getline = [&](std::string &l) {
        l.clear();
        int c;
        while ((c = fgetc(fp)) != EOF && c != '\n') l.push_back((char)c);
        return !(c == EOF && l.empty());
    };
    if (!getline(line) || sscanf(line.c_str(), "%d %d %d %d", &k, &L, &n1, &n2) != 4) {
        fclose(fp);
        set_error("%s: not a DBoW2 text vocabulary", path);
        return YGZFE_EINVAL;
    }
    std::vector<int32_t> parent(1, 0);
    std::vector<uint8_t> leaf(1, 0), desc(32, 0);
    std::vector<double> weight(1, 0.0);
    while (getline(line)) {
        const char *c = line.c_str();
        while (*c == ' ' || *c == '\t' || *c == '\r') c++;
        if (!*c) continue;
        char *end = nullptr;
        const long pid = strtol(c, &end, 10);
        c = end;
        const long isleaf = strtol(c, &end, 10);
        c = end;
        uint8_t d[32];
        for (int i = 0; i < 32; i++) {
            d[i] = (uint8_t)strtol(c, &end, 10);
            c = end;
        }
        const double w = strtod(c, &end);
        parent.push_back((int32_t)pid);
        leaf.push_back(isleaf > 0);
        desc.insert(desc.end(), d, d + 32);
        weight.push_back(w);
    }
    fclose(fp);
    return vocab_build(device, k, L, n1, n2, (int)parent.size(), parent.data(), leaf.data(), desc.data(),
                       weight.data(), out);
}

extern "C" int ygzfe_vocab_load_binary(int device, const char *path, ygzfe_vocab **out) {
    // TemplatedVocabulary::loadFromBinaryFile (TemplatedVocabulary.h:1478-1525): header
    // nb_nodes, size_node, k, L, scoring, weighting; records {int parent; u8 desc[32];
    // float weight; bool leaf}.  The reference's `while (!f.eof())` runs once more
    // after the last record with the buffer unchanged, appending a copy of the last
    // node; that copy is reproduced here.
    if (!path || !out) { set_error("invalid argument"); return YGZFE_EINVAL; }
    FILE *fp = fopen(path, "rb");
    if (!fp) { set_error("cannot open %s", path); return YGZFE_EINVAL; }
    uint32_t nb = 0, sz = 0;
    int32_t hk = 0, hL = 0, hs = 0, hw = 0;
    if (fread(&nb, 4, 1, fp) != 1 || fread(&sz, 4, 1, fp) != 1 || fread(&hk, 4, 1, fp) != 1 ||
        fread(&hL, 4, 1, fp) != 1 || fread(&hs, 4, 1, fp) != 1 || fread(&hw, 4, 1, fp) != 1 || sz < 41) {
        fclose(fp);
        set_error("%s: not a DBoW2 binary vocabulary", path);
        return YGZFE_EINVAL;
    }
    std::vector<int32_t> parent(1, 0);
    std::vector<uint8_t> leaf(1, 0), desc(32, 0), buf(sz, 0);
    std::vector<double> weight(1, 0.0);
    bool any = false;
    for (;;) {
        const bool got = fread(buf.data(), 1, sz, fp) == sz;
        if (!got && !any) break;
        int32_t pid;
        float w;
        memcpy(&pid, buf.data(), 4);
        memcpy(&w, buf.data() + 36, 4);
        parent.push_back(pid);
        desc.insert(desc.end(), buf.data() + 4, buf.data() + 36);
        weight.push_back((double)w);
        leaf.push_back(buf[40] != 0);
        any = true;
        if (!got) break;
    }
    fclose(fp);
    return vocab_build(device, hk, hL, hs, hw, (int)parent.size(), parent.data(), leaf.data(), desc.data(),
                       weight.data(), out);
}

extern "C" void ygzfe_vocab_destroy(ygzfe_vocab *v) {
    if (!v) return;
    (void)hipSetDevice(v->device);
    if (v->stream) (void)hipStreamSynchronize(v->stream), (void)hipStreamDestroy(v->stream);
    delete v;
}

extern "C" int ygzfe_vocab_info(const ygzfe_vocab *v, int *k, int *L, int *scoring, int *weighting, int *n_nodes,
                                int *n_words) {
    if (!v) { set_error("null vocabulary"); return YGZFE_EINVAL; }
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (scoring) *scoring = v->scoring;
    if (weighting) *weighting = v->weighting;
    if (n_nodes) *n_nodes = v->n_nodes;
    if (n_words) *n_words = v->n_words;
    return YGZFE_OK;
}

// one frame: host descriptors -> pinned staging -> device (one DMA) -> transform (+ vectors)
// -> one DMA of the whole result block back into pinned memory -> one synchronisation
static int bow_one(ygzfe_vocab *v, const uint8_t *desc, int n, int levelsup, bool vectors, int32_t *word,
                   double *weight, int32_t *nid, int32_t *bow_words, double *bow_values, int *n_words,
                   int32_t *fv_nodes, int32_t *fv_features, int *n_fv) {
    if (n > kBowMaxFeatures) { set_error("%d descriptors > %d per frame", n, kBowMaxFeatures); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(v->device));
    std::lock_guard<std::mutex> lk(v->mu);
    hipStream_t st = v->stream;
    const size_t N = (size_t)std::max(n, 1);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    // device block: descriptors | word, weight, node (transform) | BowVector words, values,
    // FeatureVector nodes, features, the two counts (vectors); each part 256-B aligned
    const size_t o_d = 0, o_w = al(32 * N), o_v = al(o_w + 4 * N), o_n = al(o_v + 8 * N);
    const size_t o_bw = al(o_n + 4 * N), o_bv = al(o_bw + 4 * N), o_fn = al(o_bv + 8 * N), o_ff = al(o_fn + 4 * N);
    const size_t o_c = al(o_ff + 4 * N), total = al(o_c + 16);
    YGZ_TRY(v->scratch.ensure(total));
    uint8_t *d = v->scratch.as<uint8_t>();
    int *cnt = (int *)(d + o_c);
    const size_t r0 = vectors ? o_bw : o_w, r1 = vectors ? o_c + 16 : o_n + 4 * N;  // the result block
    YGZ_TRY(v->hin.ensure(32 * N));
    YGZ_TRY(v->hout.ensure(r1 - r0));
    if (n > 0) {
        memcpy(v->hin.p, desc, 32 * (size_t)n);
        YGZ_HIP(hipMemcpyAsync(d + o_d, v->hin.p, 32 * (size_t)n, hipMemcpyHostToDevice, st));
    }
    const int nn = v->n_words > 0 ? n : 0;  // transform() returns early on an empty vocabulary
    YGZ_HIP(launch_bow_transform(v->dev(), d + o_d, 0, nullptr, nn, 1, levelsup, (int32_t *)(d + o_w),
                                 (double *)(d + o_v), (int32_t *)(d + o_n), 0, st));
    if (vectors)
        YGZ_HIP(launch_bow_vectors(nullptr, nn, 1, (int32_t *)(d + o_w), (double *)(d + o_v), (int32_t *)(d + o_n), 0,
                                   v->weighting, v->scoring, (int32_t *)(d + o_bw), (double *)(d + o_bv), cnt,
                                   (int32_t *)(d + o_fn), (int32_t *)(d + o_ff), cnt + 1, 0, st));
    if (vectors || nn > 0) YGZ_HIP(hipMemcpyAsync(v->hout.p, d + r0, r1 - r0, hipMemcpyDeviceToHost, st));
    YGZ_HIP(hipStreamSynchronize(st));
    const uint8_t *h = v->hout.as<uint8_t>() - r0;  // h + o_x: part o_x of the block
    if (!vectors) {
        if (nn > 0) {
            memcpy(word, h + o_w, 4 * (size_t)n);
            memcpy(weight, h + o_v, 8 * (size_t)n);
            memcpy(nid, h + o_n, 4 * (size_t)n);
        }
        return YGZFE_OK;
    }
    const int *hc = (const int *)(h + o_c);
    *n_words = hc[0];
    *n_fv = hc[1];
    if (hc[0] > 0) {
        memcpy(bow_words, h + o_bw, 4 * (size_t)hc[0]);
        memcpy(bow_values, h + o_bv, 8 * (size_t)hc[0]);
    }
    if (hc[1] > 0) {
        memcpy(fv_nodes, h + o_fn, 4 * (size_t)hc[1]);
        memcpy(fv_features, h + o_ff, 4 * (size_t)hc[1]);
    }
    return YGZFE_OK;
}

extern "C" int ygzfe_bow_transform(ygzfe_vocab *v, const uint8_t *desc, int n, int levelsup, int32_t *word,
                                   double *weight, int32_t *nid) {
    if (!v || n < 0 || (n > 0 && (!desc || !word || !weight || !nid))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (n > 0 && v->n_words == 0) { set_error("empty vocabulary"); return YGZFE_EINVAL; }
    if (n == 0) return YGZFE_OK;
    return bow_one(v, desc, n, levelsup, false, word, weight, nid, nullptr, nullptr, nullptr, nullptr, nullptr,
                   nullptr);
}

extern "C" int ygzfe_compute_bow(ygzfe_vocab *v, const uint8_t *desc, int n, int levelsup, int32_t *bow_words,
                                 double *bow_values, int *n_words, int32_t *fv_nodes, int32_t *fv_features,
                                 int *n_fv) {
    if (!v || n < 0 || !n_words || !n_fv ||
        (n > 0 && (!desc || !bow_words || !bow_values || !fv_nodes || !fv_features))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    *n_words = 0;
    *n_fv = 0;
    if (n == 0) return YGZFE_OK;
    return bow_one(v, desc, n, levelsup, true, nullptr, nullptr, nullptr, bow_words, bow_values, n_words, fv_nodes,
                   fv_features, n_fv);
}

extern "C" int ygzfe_batch_compute_bow(ygzfe_batch *b, ygzfe_vocab *v, int n_frames, int levelsup,
                                       int32_t *d_bow_words, double *d_bow_values, int *d_n_words,
                                       int32_t *d_fv_nodes, int32_t *d_fv_features, int *d_n_fv, void *stream) {
    if (!b || !v || n_frames < 0 ||
        (n_frames > 0 && (!d_bow_words || !d_bow_values || !d_n_words || !d_fv_nodes || !d_fv_features || !d_n_fv))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (n_frames > b->maxF) { set_error("n_frames %d > batch capacity %d", n_frames, b->maxF); return YGZFE_EINVAL; }
    if (b->device != v->device) { set_error("vocabulary and batch live on different devices"); return YGZFE_EINVAL; }
    if (n_frames == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(b->device));
    hipStream_t st = stream ? (hipStream_t)stream : b->stream;
    const Plan &P = b->plan->hp();
    if (P.kp_cap > kBowMaxFeatures) { set_error("kp_cap %d > %d", P.kp_cap, kBowMaxFeatures); return YGZFE_EINVAL; }
    const size_t cells = (size_t)n_frames * P.kp_cap;
    YGZ_TRY(b->bow_word.ensure(4 * cells));
    YGZ_TRY(b->bow_weight.ensure(8 * cells));
    YGZ_TRY(b->bow_nid.ensure(4 * cells));
    if (v->n_words == 0) {  // transform() clears the vectors and returns
        YGZ_HIP(hipMemsetAsync(d_n_words, 0, 4 * (size_t)n_frames, st));
        YGZ_HIP(hipMemsetAsync(d_n_fv, 0, 4 * (size_t)n_frames, st));
        return YGZFE_OK;
    }
    YGZ_HIP(launch_bow_transform(v->dev(), b->ws.desc.as<uint8_t>(), (size_t)P.kp_cap * 32, b->ws.counts.as<int>(),
                                 P.kp_cap, n_frames, levelsup, b->bow_word.as<int32_t>(), b->bow_weight.as<double>(),
                                 b->bow_nid.as<int32_t>(), P.kp_cap, st));
    YGZ_HIP(launch_bow_vectors(b->ws.counts.as<int>(), 0, n_frames, b->bow_word.as<int32_t>(),
                               b->bow_weight.as<double>(), b->bow_nid.as<int32_t>(), P.kp_cap, v->weighting,
                               v->scoring, d_bow_words, d_bow_values, d_n_words, d_fv_nodes, d_fv_features, d_n_fv,
                               P.kp_cap, st));
    return YGZFE_OK;
}

// --------------------------------------------------------------------------
// Undistortion (Frame.cc:775-790)
struct ygzfe_undistort {
    int device = 0;
    int W = 0, H = 0;
    hipStream_t stream = nullptr;
    DevBuf map1, map2, boxes, raw;  // boxes: per-tile source boxes; raw: host-frame staging
    int max_box = 0;                // largest LDS-staged box (bytes)
    bool any_large = false;         // some tile's box exceeds the LDS stage (global-gather kernel)
};

extern "C" int ygzfe_undistort_create(int device, const ygzfe_camera *K, const float *dist, int ndist, int width,
                                      int height, ygzfe_undistort **out) {
    if (!K || !out || (ndist > 0 && !dist) || ndist < 0 || ndist > 12 || width < 2 || height < 2 ||
        (size_t)width * height > (1u << 30)) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (width > 32767 || height > 32767) { set_error("image too large for CV_16SC2 maps"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(device));
    std::unique_ptr<ygzfe_undistort> u(new ygzfe_undistort());
    u->device = device;
    u->W = width;
    u->H = height;
    const size_t n = (size_t)width * height;
    YGZ_TRY(u->map1.ensure(4 * n));
    YGZ_TRY(u->map2.ensure(2 * n));
    YGZ_TRY(u->boxes.ensure(16 * (size_t)remap_tiles(width, height)));
    YGZ_HIP(hipStreamCreateWithFlags(&u->stream, hipStreamNonBlocking));
    const float cam[4] = {K->fx, K->fy, K->cx, K->cy};
    YGZ_HIP(launch_undistort_map(cam, dist, ndist, width, height, u->map1.as<int16_t>(), u->map2.as<uint16_t>(),
                                 u->stream));
    YGZ_HIP(launch_remap_boxes(width, height, u->map1.as<int16_t>(), u->boxes.p, u->stream));
    std::vector<int32_t> boxes(4 * (size_t)remap_tiles(width, height));
    YGZ_HIP(hipMemcpyAsync(boxes.data(), u->boxes.p, 4 * boxes.size(), hipMemcpyDeviceToHost, u->stream));
    YGZ_HIP(hipStreamSynchronize(u->stream));
    for (size_t i = 0; i < boxes.size(); i += 4)
        if (boxes[i + 3] > 0) u->max_box = std::max(u->max_box, boxes[i + 2] * boxes[i + 3]);
        else if (boxes[i + 3] < 0) u->any_large = true;
    *out = u.release();
    return YGZFE_OK;
}

extern "C" void ygzfe_undistort_destroy(ygzfe_undistort *u) {
    if (!u) return;
    (void)hipSetDevice(u->device);
    (void)hipStreamSynchronize(u->stream);
    (void)hipStreamDestroy(u->stream);
    delete u;
}

extern "C" int ygzfe_undistort_maps(const ygzfe_undistort *u, int16_t *map1, uint16_t *map2) {
    if (!u) { set_error("null handle"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(u->device));
    const size_t n = (size_t)u->W * u->H;
    if (map1) YGZ_HIP(hipMemcpy(map1, u->map1.p, 4 * n, hipMemcpyDeviceToHost));
    if (map2) YGZ_HIP(hipMemcpy(map2, u->map2.p, 2 * n, hipMemcpyDeviceToHost));
    return YGZFE_OK;
}

extern "C" int ygzfe_undistort_apply_device(const ygzfe_undistort *u, const uint8_t *d_src, size_t src_pitch,
                                            int src_stride, uint8_t *d_dst, size_t dst_pitch, int dst_stride,
                                            int n_images, void *stream) {
    if (!u || n_images < 0 || (n_images > 0 && (!d_src || !d_dst)) || src_stride < u->W || dst_stride < u->W ||
        (n_images > 1 && (src_pitch < (size_t)src_stride * u->H || dst_pitch < (size_t)dst_stride * u->H)) ||
        n_images > 65535) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (n_images == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(u->device));
    hipStream_t st = stream ? (hipStream_t)stream : u->stream;
    YGZ_HIP(launch_remap_linear(d_src, src_pitch, u->W, u->H, src_stride, u->map1.as<int16_t>(),
                                u->map2.as<uint16_t>(), u->boxes.p, u->max_box, u->any_large, d_dst, dst_pitch,
                                dst_stride, n_images, st));
    if (!stream) YGZ_HIP(hipStreamSynchronize(st));
    return YGZFE_OK;
}

extern "C" int ygzfe_undistort_apply_f32_device(const ygzfe_undistort *u, const float *d_src, size_t src_pitch,
                                                int src_stride, float *d_dst, size_t dst_pitch, int dst_stride,
                                                int n_images, void *stream) {
    if (!u || n_images < 0 || (n_images > 0 && (!d_src || !d_dst)) || src_stride < u->W || dst_stride < u->W ||
        (n_images > 1 && (src_pitch < (size_t)src_stride * u->H || dst_pitch < (size_t)dst_stride * u->H)) ||
        n_images > 65535) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (n_images == 0) return YGZFE_OK;
    YGZ_TRY(ensure_device(u->device));
    hipStream_t st = stream ? (hipStream_t)stream : u->stream;
    YGZ_HIP(launch_remap_f32(d_src, src_pitch, u->W, u->H, src_stride, u->map1.as<int16_t>(), u->map2.as<uint16_t>(),
                             d_dst, dst_pitch, dst_stride, n_images, st));
    if (!stream) YGZ_HIP(hipStreamSynchronize(st));
    return YGZFE_OK;
}

// host image in, host image out: one H2D, the remap, one D2H (leased staging)
static int undistort_host(const ygzfe_undistort *u, const void *src, int src_stride, void *dst, int dst_stride,
                          int esize) {
    if (!u || !src || !dst || src_stride < u->W || dst_stride < u->W) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    YGZ_TRY(ensure_device(u->device));
    StagingLease S;
    YGZ_TRY(S.acquire(u->device));
    const size_t row = (size_t)u->W * esize, img = row * u->H, o_d = align16(img);
    YGZ_TRY(S->hin.ensure(img));
    YGZ_TRY(S->hout.ensure(img));
    YGZ_TRY(S->dev.ensure(o_d + img));
    uint8_t *h = S->hin.as<uint8_t>(), *d = S->dev.as<uint8_t>();
    for (int y = 0; y < u->H; y++)
        memcpy(h + (size_t)y * row, static_cast<const uint8_t *>(src) + (size_t)y * src_stride * esize, row);
    YGZ_HIP(hipMemcpyAsync(d, h, img, hipMemcpyHostToDevice, S->stream));
    if (esize == 4)
        YGZ_HIP(launch_remap_f32(reinterpret_cast<const float *>(d), 0, u->W, u->H, u->W, u->map1.as<int16_t>(),
                                 u->map2.as<uint16_t>(), reinterpret_cast<float *>(d + o_d), 0, u->W, 1, S->stream));
    else
        YGZ_HIP(launch_remap_linear(d, 0, u->W, u->H, u->W, u->map1.as<int16_t>(), u->map2.as<uint16_t>(), u->boxes.p,
                                    u->max_box, u->any_large, d + o_d, 0, u->W, 1, S->stream));
    YGZ_HIP(hipMemcpyAsync(S->hout.p, d + o_d, img, hipMemcpyDeviceToHost, S->stream));
    YGZ_HIP(hipStreamSynchronize(S->stream));
    for (int y = 0; y < u->H; y++)
        memcpy(static_cast<uint8_t *>(dst) + (size_t)y * dst_stride * esize, S->hout.as<uint8_t>() + (size_t)y * row,
               row);
    return YGZFE_OK;
}

extern "C" int ygzfe_undistort_image(const ygzfe_undistort *u, const uint8_t *src, int src_stride, uint8_t *dst,
                                     int dst_stride) {
    return undistort_host(u, src, src_stride, dst, dst_stride, 1);
}

extern "C" int ygzfe_undistort_depth(const ygzfe_undistort *u, const float *src, int src_stride, float *dst,
                                     int dst_stride) {
    return undistort_host(u, src, src_stride, dst, dst_stride, 4);
}

extern "C" int ygzfe_compute_pyramid_undistorted(ygzfe_extractor *ex, ygzfe_frame *f, ygzfe_undistort *u,
                                                 const uint8_t *img, int stride) {
    if (!ex || !f || !u || !img || stride < f->W) { set_error("invalid argument"); return YGZFE_EINVAL; }
    if (u->W != f->W || u->H != f->H || u->device != ex->device) {
        set_error("undistort maps are %dx%d on device %d, frame is %dx%d on device %d", u->W, u->H, u->device, f->W,
                  f->H, ex->device);
        return YGZFE_EINVAL;
    }
    YGZ_TRY(ensure_device(ex->device));
    std::lock_guard<std::mutex> lk(ex->mu);
    const size_t n = (size_t)f->W * f->H;
    YGZ_TRY(u->raw.ensure(n));
    YGZ_HIP(hipMemcpy2DAsync(u->raw.p, f->W, img, stride, f->W, f->H, hipMemcpyHostToDevice, ex->stream));
    YGZ_HIP(launch_remap_linear(u->raw.as<uint8_t>(), n, f->W, f->H, f->W, u->map1.as<int16_t>(),
                                u->map2.as<uint16_t>(), u->boxes.p, u->max_box, u->any_large, f->pyr.as<uint8_t>(),
                                n, f->W, 1, ex->stream));
    YGZ_TRY(pyramid_from_level0(f, ex->stream));
    YGZ_HIP(hipStreamSynchronize(ex->stream));
    return YGZFE_OK;
}

static int batch_undistort_check(const ygzfe_batch *b, const ygzfe_undistort *u, int n_frames) {
    if (!b || !u || n_frames < 0 || n_frames > b->maxF) { set_error("invalid argument"); return YGZFE_EINVAL; }
    const Plan &P = b->plan->hp();
    if (u->W != P.W || u->H != P.H || u->device != b->device) {
        set_error("undistort maps are %dx%d on device %d, batch is %dx%d on device %d", u->W, u->H, u->device, P.W,
                  P.H, b->device);
        return YGZFE_EINVAL;
    }
    return YGZFE_OK;
}

extern "C" int ygzfe_batch_undistort_device(ygzfe_batch *b, const ygzfe_undistort *u, const uint8_t *d_raw,
                                            size_t raw_pitch, int n_frames, void *stream) {
    YGZ_TRY(batch_undistort_check(b, u, n_frames));
    if (n_frames == 0) return YGZFE_OK;
    const Plan &P = b->plan->hp();
    if (!d_raw || (n_frames > 1 && raw_pitch < (size_t)P.W * P.H)) { set_error("invalid raw frames"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(b->device));
    hipStream_t st = stream ? (hipStream_t)stream : b->stream;
    YGZ_HIP(launch_remap_linear(d_raw, raw_pitch, P.W, P.H, P.W, u->map1.as<int16_t>(), u->map2.as<uint16_t>(),
                                u->boxes.p, u->max_box, u->any_large, b->pyr.as<uint8_t>(), P.pyr_bytes, P.W,
                                n_frames, st));
    return YGZFE_OK;
}

extern "C" int ygzfe_batch_upload_undistorted(ygzfe_batch *b, ygzfe_undistort *u, const uint8_t *frames,
                                              int n_frames) {
    YGZ_TRY(batch_undistort_check(b, u, n_frames));
    if (n_frames == 0) return YGZFE_OK;
    if (!frames) { set_error("null frames"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(b->device));
    const Plan &P = b->plan->hp();
    const size_t n = (size_t)P.W * P.H;
    YGZ_TRY(u->raw.ensure(n * n_frames));
    YGZ_HIP(hipMemcpyAsync(u->raw.p, frames, n * n_frames, hipMemcpyHostToDevice, b->stream));
    YGZ_HIP(launch_remap_linear(u->raw.as<uint8_t>(), n, P.W, P.H, P.W, u->map1.as<int16_t>(),
                                u->map2.as<uint16_t>(), u->boxes.p, u->max_box, u->any_large, b->pyr.as<uint8_t>(),
                                P.pyr_bytes, P.W, n_frames, b->stream));
    YGZ_HIP(hipStreamSynchronize(b->stream));
    return YGZFE_OK;
}

// --------------------------------------------------------------------------
// ORBmatcher searches (match.hip): the searched frame's state on the device,
// one packed H2D of the queries, two launches, one packed D2H of the results.
struct ygzfe_match_frame {
    int device = 0;
    hipStream_t stream = nullptr;
    int n = 0;
    bool has_uright = false;
    ygzfe_bounds bounds{0.f, 0.f, 0.f, 0.f};
    float inv_w = 0.f, inv_h = 0.f;
    DevBuf kps, desc, uright, cell;
    std::vector<ygzfe_kp> host_kps;  // angles / octaves / positions the host-side query building reads
    int last_rescans = 0;            // queries of the last search whose top-K list the skips exhausted
    int last_passes = -1;            // parallel-resolve passes of the last search (-1: serial replay)
    // per-call staging: page-locked, one DMA per direction; ev_in = the last H2D out of
    // hin / hset (the next call refills them only after it)
    DevBuf in, out, scratch;
    HostBuf hin, hout, hset;
    hipEvent_t ev_in = nullptr, ev_set = nullptr;
    // recorded on `stream` once the frame's keypoints, descriptors and grid are on the
    // device: a search on another frame's stream that reads this frame's descriptors as
    // its queries (SearchForInitialization, SearchByBoW) waits for it
    hipEvent_t ev_ready = nullptr;
};

namespace {

constexpr int kMatchTopK = 32;  // match.hip kTopList (J.topk stride)
constexpr int kMatchCells = 64 * 48;  // FRAME_GRID_COLS x ROWS

struct Arena {
    size_t off = 0;
    size_t take(size_t bytes) {
        const size_t o = off;
        off = (off + bytes + 255) & ~(size_t)255;
        return o;
    }
};

int match_frame_finish(ygzfe_match_frame *f, const ygzfe_bounds *bounds) {
    f->bounds = *bounds;
    // Frame.cc:296-297
    f->inv_w = (float)64 / (float)(bounds->max_x - bounds->min_x);
    f->inv_h = (float)48 / (float)(bounds->max_y - bounds->min_y);
    // cell[n] | cell ends [64 * 48] | keypoints by cell u16[n]
    YGZ_TRY(f->cell.ensure(sizeof(int32_t) * ((size_t)f->n + kMatchCells) + sizeof(uint16_t) * (size_t)f->n + 16));
    YGZ_HIP(launch_match_cells(f->kps.as<ygzfe_kp>(), f->n, bounds->min_x, bounds->min_y, f->inv_w, f->inv_h,
                               f->cell.as<int32_t>(), f->cell.as<int32_t>() + f->n,
                               reinterpret_cast<uint16_t *>(f->cell.as<int32_t>() + f->n + kMatchCells), f->stream));
    // no host synchronisation: a search on this frame runs on f->stream after the grid;
    // one that reads this frame's descriptors from another stream waits on ev_ready
    if (!f->ev_ready) YGZ_HIP(hipEventCreateWithFlags(&f->ev_ready, hipEventDisableTiming));
    YGZ_HIP(hipEventRecord(f->ev_ready, f->stream));
    return YGZFE_OK;
}

// Run one search problem: the job's host-side arrays are staged into one H2D
// copy; outputs come back in one D2H copy.
struct MatchCall {
    ygzfe_match_frame *train;
    std::vector<ygzfe_match_query> q;
    const uint8_t *qdesc_host = nullptr;  // [n_qdesc][32] (host) or
    const uint8_t *qdesc_dev = nullptr;   // device descriptors (INIT / BoW: a match frame's)
    const ygzfe_match_frame *qframe = nullptr;  // the match frame that owns qdesc_dev
    int n_qdesc = 0;
    std::vector<int32_t> qid, cand_ptr;
    const int32_t *cand_host = nullptr;
    int n_cand = 0;
    const uint8_t *blocked_host = nullptr;
    int mode = 0, th_dist = 100, check_ori = 0;
    float nnratio = 0.6f;
    // outputs
    int32_t *train_out = nullptr, *query_out = nullptr;
    int nmatches = 0;
};

int run_match(MatchCall &c) {
    ygzfe_match_frame *f = c.train;
    const int nq = (int)c.q.size(), n = f->n;
    if (n > 65535) { set_error("match frame holds %d keypoints (<= 65535 supported)", n); return YGZFE_EINVAL; }
    if (c.mode == YGZFE_MATCH_INIT && (n > 16384 || nq > 32767)) {
        set_error("SearchForInitialization: %d x %d keypoints exceed 32767 x 16384", nq, n);
        return YGZFE_EINVAL;
    }
    YGZ_TRY(ensure_device(f->device));
    hipStream_t st = f->stream;
    // query descriptors of another match frame: uploaded on that frame's stream
    if (c.qframe && c.qframe != f && c.qframe->ev_ready) YGZ_HIP(hipStreamWaitEvent(st, c.qframe->ev_ready, 0));
    // device input layout
    Arena ai;
    const size_t o_q = ai.take(sizeof(ygzfe_match_query) * (size_t)std::max(nq, 1));
    const size_t o_qd = c.qdesc_host ? ai.take((size_t)32 * std::max(c.n_qdesc, 1)) : 0;
    const size_t o_qid = c.qid.empty() ? 0 : ai.take(sizeof(int32_t) * c.qid.size());
    const size_t o_cp = c.cand_ptr.empty() ? 0 : ai.take(sizeof(int32_t) * c.cand_ptr.size());
    const size_t o_c = c.cand_host ? ai.take(sizeof(int32_t) * (size_t)std::max(c.n_cand, 1)) : 0;
    const size_t o_bl = c.blocked_host ? ai.take((size_t)std::max(n, 1)) : 0;
    // device outputs / scratch
    Arena ao;
    const size_t o_tout = ao.take(sizeof(int32_t) * (size_t)std::max(n, 1));
    const size_t o_qout = ao.take(sizeof(int32_t) * (size_t)std::max(nq, 1));
    const size_t o_nm = ao.take(4 * sizeof(int32_t));
    const size_t out_bytes = ao.off;
    const size_t o_topk = ao.take(sizeof(uint64_t) * kMatchTopK * (size_t)std::max(nq, 1));
    const size_t o_ncand = ao.take(sizeof(int32_t) * (size_t)std::max(nq, 1));
    const size_t o_push = ao.take(sizeof(int32_t) * (size_t)std::max(nq, 1));
    const size_t o_qang = ao.take(sizeof(float) * (size_t)std::max(nq, 1));
    YGZ_TRY(f->out.ensure(ao.off));
    uint8_t *dout = f->out.as<uint8_t>();
    // The inputs stay in page-locked host memory that the kernels read directly (one
    // pass in k_match_topk, which copies what the decisions need into HBM): no H2D
    // copy and no copy-to-kernel dependency on the stream.  The previous call
    // synchronised its stream, so the staging is free.
    YGZ_TRY(f->hin.ensure(ai.off));
    uint8_t *h = f->hin.as<uint8_t>(), *din = nullptr;
    YGZ_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&din), h, 0));
    MatchJob J;
    memset(&J, 0, sizeof(J));
    J.kps = f->kps.as<ygzfe_kp>();
    J.desc = f->desc.as<uint8_t>();
    J.u_right = f->has_uright ? f->uright.as<float>() : nullptr;
    J.cell = f->cell.as<int32_t>();
    J.cend = J.cell + n;
    J.cidx = reinterpret_cast<const uint16_t *>(J.cend + kMatchCells);
    J.n_train = n;
    J.min_x = f->bounds.min_x;
    J.min_y = f->bounds.min_y;
    J.inv_w = f->inv_w;
    J.inv_h = f->inv_h;
    J.q = reinterpret_cast<const ygzfe_match_query *>(din + o_q);
    J.qdesc = c.qdesc_host ? din + o_qd : c.qdesc_dev;
    J.qid = c.qid.empty() ? nullptr : reinterpret_cast<const int32_t *>(din + o_qid);
    J.nq = nq;
    J.cand_ptr = c.cand_ptr.empty() ? nullptr : reinterpret_cast<const int32_t *>(din + o_cp);
    J.cand = c.cand_host ? reinterpret_cast<const int32_t *>(din + o_c) : nullptr;
    J.blocked0 = c.blocked_host ? din + o_bl : nullptr;
    J.topk = reinterpret_cast<uint64_t *>(dout + o_topk);
    J.ncand = reinterpret_cast<int32_t *>(dout + o_ncand);
    J.qangle = reinterpret_cast<float *>(dout + o_qang);
    J.train_out = reinterpret_cast<int32_t *>(dout + o_tout);
    J.query_out = reinterpret_cast<int32_t *>(dout + o_qout);
    J.pushes = reinterpret_cast<int32_t *>(dout + o_push);
    J.nmatches = reinterpret_cast<int32_t *>(dout + o_nm);
    if (nq) memcpy(h + o_q, c.q.data(), sizeof(ygzfe_match_query) * nq);
    if (c.qdesc_host && c.n_qdesc) memcpy(h + o_qd, c.qdesc_host, (size_t)32 * c.n_qdesc);
    if (!c.qid.empty()) memcpy(h + o_qid, c.qid.data(), sizeof(int32_t) * c.qid.size());
    if (!c.cand_ptr.empty()) memcpy(h + o_cp, c.cand_ptr.data(), sizeof(int32_t) * c.cand_ptr.size());
    if (c.cand_host && c.n_cand) memcpy(h + o_c, c.cand_host, sizeof(int32_t) * c.n_cand);
    if (c.blocked_host && n) memcpy(h + o_bl, c.blocked_host, (size_t)n);
    // YGZFE_MATCH_PASSES=0 selects the serial replay (tests run both paths)
    const char *ev = getenv("YGZFE_MATCH_PASSES");
    const int max_passes = ev ? atoi(ev) : 1;
    YGZ_TRY(f->hout.ensure(out_bytes));
    const bool direct = match_resolves(n, nq, c.mode, max_passes);
    if (direct) {  // k_match_resolve writes each output once, straight into page-locked host memory
        uint8_t *hod = nullptr;
        YGZ_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&hod), f->hout.p, 0));
        J.train_out = reinterpret_cast<int32_t *>(hod + o_tout);
        J.nmatches = reinterpret_cast<int32_t *>(hod + o_nm);
    }
    YGZ_HIP(launch_match(J, c.mode, c.th_dist, c.check_ori, c.nnratio, max_passes, st));
    if (!direct) YGZ_HIP(hipMemcpyAsync(f->hout.p, dout, out_bytes, hipMemcpyDeviceToHost, st));
    YGZ_HIP(hipStreamSynchronize(st));
    const uint8_t *ho = f->hout.as<uint8_t>();
    if (c.train_out && n) memcpy(c.train_out, ho + o_tout, sizeof(int32_t) * n);
    if (c.query_out && nq) memcpy(c.query_out, ho + o_qout, sizeof(int32_t) * nq);
    memcpy(&c.nmatches, ho + o_nm, sizeof(int32_t));
    memcpy(&f->last_rescans, ho + o_nm + 4, sizeof(int32_t));
    memcpy(&f->last_passes, ho + o_nm + 8, sizeof(int32_t));
    if (max_passes > 0 && f->last_passes < 0 && c.mode != YGZFE_MATCH_INIT && nq > 0 && nq <= 4096 &&
        resolve_fits(n, nq)) {
        set_error("match resolve did not reach its fixed point within nq + 2 passes (internal error)");
        return YGZFE_EHIP;
    }
    return YGZFE_OK;
}

}  // namespace

extern "C" int ygzfe_match_frame_create(int device, ygzfe_match_frame **out) {
    if (!out) { set_error("null out"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(device));
    std::unique_ptr<ygzfe_match_frame> f(new ygzfe_match_frame());
    f->device = device;
    YGZ_HIP(hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking));
    *out = f.release();
    return YGZFE_OK;
}

extern "C" void ygzfe_match_frame_destroy(ygzfe_match_frame *f) {
    if (!f) return;
    (void)hipSetDevice(f->device);
    if (f->stream) (void)hipStreamSynchronize(f->stream), (void)hipStreamDestroy(f->stream);
    if (f->ev_in) (void)hipEventDestroy(f->ev_in);
    if (f->ev_set) (void)hipEventDestroy(f->ev_set);
    if (f->ev_ready) (void)hipEventDestroy(f->ev_ready);
    delete f;
}

extern "C" int ygzfe_match_frame_stats(const ygzfe_match_frame *f, int *rescans) {
    if (!f || !rescans) { set_error("invalid argument"); return YGZFE_EINVAL; }
    *rescans = f->last_rescans;
    return YGZFE_OK;
}

extern "C" int ygzfe_match_frame_resolve_stats(const ygzfe_match_frame *f, int *passes) {
    if (!f || !passes) { set_error("invalid argument"); return YGZFE_EINVAL; }
    *passes = f->last_passes;
    return YGZFE_OK;
}

extern "C" int ygzfe_match_frame_set(ygzfe_match_frame *f, const ygzfe_kp *kps, const uint8_t *desc, int n,
                                     const float *u_right, const ygzfe_bounds *bounds) {
    if (!f || !bounds || n < 0 || n > 65535 || (n > 0 && (!kps || !desc))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (!(bounds->max_x > bounds->min_x) || !(bounds->max_y > bounds->min_y)) {
        set_error("empty image bounds");
        return YGZFE_EINVAL;
    }
    YGZ_TRY(ensure_device(f->device));
    f->n = n;
    f->host_kps.assign(kps, kps + n);
    YGZ_TRY(f->kps.ensure(sizeof(ygzfe_kp) * (size_t)std::max(n, 1)));
    YGZ_TRY(f->desc.ensure((size_t)32 * std::max(n, 1)));
    f->has_uright = u_right != nullptr;
    if (u_right) YGZ_TRY(f->uright.ensure(sizeof(float) * (size_t)std::max(n, 1)));
    if (n) {  // keypoints, descriptors (and u_right) through page-locked staging: async DMAs
        const size_t kb = sizeof(ygzfe_kp) * (size_t)n, db = (size_t)32 * n, ub = u_right ? sizeof(float) * n : 0;
        if (f->ev_set) YGZ_HIP(hipEventSynchronize(f->ev_set));  // the previous frame's DMA out of hset
        // test hook (tests/test_gpu_match_search.py): hold this frame's stream before its
        // upload, so a search on another frame's stream that skipped the ev_ready wait
        // would read descriptors that are not there yet
        if (const char *hold = getenv("YGZFE_DEBUG_SET_HOLD_US")) YGZ_HIP(launch_hold_us(atoi(hold), f->stream));
        YGZ_TRY(f->hset.ensure(kb + db + ub));
        uint8_t *hs = f->hset.as<uint8_t>();
        memcpy(hs, kps, kb);
        memcpy(hs + kb, desc, db);
        if (ub) memcpy(hs + kb + db, u_right, ub);
        YGZ_HIP(hipMemcpyAsync(f->kps.p, hs, kb, hipMemcpyHostToDevice, f->stream));
        YGZ_HIP(hipMemcpyAsync(f->desc.p, hs + kb, db, hipMemcpyHostToDevice, f->stream));
        if (ub) YGZ_HIP(hipMemcpyAsync(f->uright.p, hs + kb + db, ub, hipMemcpyHostToDevice, f->stream));
        if (!f->ev_set) YGZ_HIP(hipEventCreateWithFlags(&f->ev_set, hipEventDisableTiming));
        YGZ_HIP(hipEventRecord(f->ev_set, f->stream));
    }
    return match_frame_finish(f, bounds);
}

extern "C" int ygzfe_match_frame_from_batch(ygzfe_match_frame *f, ygzfe_batch *b, int frame,
                                            const ygzfe_bounds *bounds) {
    if (!f || !b || !bounds || frame < 0 || frame >= b->maxF) { set_error("invalid argument"); return YGZFE_EINVAL; }
    if (f->device != b->device) { set_error("match frame and batch on different devices"); return YGZFE_EINVAL; }
    YGZ_TRY(ensure_device(f->device));
    const Plan &P = b->plan->hp();
    YGZ_TRY(batch_wait(b));  // the batch's extraction may run on caller streams
    int n = 0;
    YGZ_HIP(hipMemcpy(&n, b->ws.counts.as<int>() + frame, sizeof(int), hipMemcpyDeviceToHost));
    f->n = n;
    YGZ_TRY(f->kps.ensure(sizeof(ygzfe_kp) * (size_t)std::max(n, 1)));
    YGZ_TRY(f->desc.ensure((size_t)32 * std::max(n, 1)));
    f->host_kps.resize(n);
    if (n) {
        YGZ_HIP(hipMemcpyAsync(f->kps.p, b->ws.kps.as<ygzfe_kp>() + (size_t)frame * P.kp_cap, sizeof(ygzfe_kp) * n,
                               hipMemcpyDeviceToDevice, f->stream));
        YGZ_HIP(hipMemcpyAsync(f->desc.p, b->ws.desc.as<uint8_t>() + (size_t)frame * P.kp_cap * 32, (size_t)32 * n,
                               hipMemcpyDeviceToDevice, f->stream));
        YGZ_HIP(hipMemcpyAsync(f->host_kps.data(), f->kps.p, sizeof(ygzfe_kp) * n, hipMemcpyDeviceToHost, f->stream));
    }
    f->has_uright = false;
    YGZ_TRY(match_frame_finish(f, bounds));
    // host_kps (read by the host when this frame is a SearchForInitialization / BoW query
    // frame) arrives by the async D2H above
    YGZ_HIP(hipStreamSynchronize(f->stream));
    return YGZFE_OK;
}

extern "C" int ygzfe_search_projection_best(ygzfe_match_frame *cur, const ygzfe_match_query *q, const uint8_t *q_desc,
                                            int nq, const uint8_t *train_blocked, int th_dist, int check_ori,
                                            int32_t *train_match, int *nmatches) {
    if (!cur || nq < 0 || (nq > 0 && (!q || !q_desc)) || !train_match || !nmatches) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    MatchCall c;
    c.train = cur;
    c.q.assign(q, q + nq);
    c.qdesc_host = q_desc;
    c.n_qdesc = nq;
    c.blocked_host = train_blocked;
    c.mode = YGZFE_MATCH_BEST;
    c.th_dist = th_dist;
    c.check_ori = check_ori;
    c.train_out = train_match;
    YGZ_TRY(run_match(c));
    *nmatches = c.nmatches;
    return YGZFE_OK;
}

extern "C" int ygzfe_search_projection_ratio(ygzfe_match_frame *F, const ygzfe_match_query *q, const uint8_t *q_desc,
                                             int nq, const uint8_t *train_blocked, float nnratio, int32_t *train_match,
                                             int *nmatches) {
    if (!F || nq < 0 || (nq > 0 && (!q || !q_desc)) || !train_match || !nmatches) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    MatchCall c;
    c.train = F;
    c.q.assign(q, q + nq);
    c.qdesc_host = q_desc;
    c.n_qdesc = nq;
    c.blocked_host = train_blocked;
    c.mode = YGZFE_MATCH_RATIO;
    c.nnratio = nnratio;
    c.train_out = train_match;
    YGZ_TRY(run_match(c));
    *nmatches = c.nmatches;
    return YGZFE_OK;
}

extern "C" int ygzfe_search_for_initialization(ygzfe_match_frame *F1, ygzfe_match_frame *F2, float *prev_matched,
                                               int window_size, float nnratio, int check_ori, int32_t *matches12,
                                               int *nmatches) {
    if (!F1 || !F2 || (F1->n > 0 && (!prev_matched || !matches12)) || !nmatches) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (F1->device != F2->device) { set_error("frames on different devices"); return YGZFE_EINVAL; }
    // ORBmatcher.cc:388-398: queries = F1's keypoints, level-0 only, window at vbPrevMatched
    MatchCall c;
    c.train = F2;
    c.q.resize(F1->n);
    for (int i = 0; i < F1->n; i++) {
        ygzfe_match_query &Q = c.q[i];
        const ygzfe_kp &kp = F1->host_kps[i];
        Q.u = prev_matched[2 * i];
        Q.v = prev_matched[2 * i + 1];
        Q.radius = (float)window_size;
        Q.u_right = 0.f;
        Q.min_level = kp.octave;
        Q.max_level = kp.octave;
        Q.angle = kp.angle;
        Q.flags = kp.octave > 0 ? 0 : YGZFE_MQ_VALID;
    }
    c.qdesc_dev = F1->desc.as<uint8_t>();
    c.qframe = F1;
    c.mode = YGZFE_MATCH_INIT;
    c.nnratio = nnratio;
    c.check_ori = check_ori;
    c.query_out = matches12;
    YGZ_TRY(run_match(c));
    *nmatches = c.nmatches;
    // :472-475 update prev matched
    for (int i = 0; i < F1->n; i++)
        if (matches12[i] >= 0) {
            prev_matched[2 * i] = F2->host_kps[matches12[i]].x;
            prev_matched[2 * i + 1] = F2->host_kps[matches12[i]].y;
        }
    return YGZFE_OK;
}

extern "C" int ygzfe_search_by_bow(ygzfe_match_frame *kf, ygzfe_match_frame *F, const uint8_t *kf_usable,
                                   int n_kf_nodes, const int32_t *kf_nodes, const int32_t *kf_ptr,
                                   const int32_t *kf_feats, int n_f_nodes, const int32_t *f_nodes,
                                   const int32_t *f_ptr, const int32_t *f_feats, float nnratio, int check_ori,
                                   int32_t *f_match, int *nmatches) {
    if (!kf || !F || !kf_usable || !f_match || !nmatches || n_kf_nodes < 0 || n_f_nodes < 0 ||
        (n_kf_nodes > 0 && (!kf_nodes || !kf_ptr || !kf_feats)) || (n_f_nodes > 0 && (!f_nodes || !f_ptr || !f_feats))) {
        set_error("invalid argument");
        return YGZFE_EINVAL;
    }
    if (kf->device != F->device) { set_error("frames on different devices"); return YGZFE_EINVAL; }
    // ORBmatcher.cc:170-243: walk the two node-sorted FeatureVectors; every KF feature of
    // a shared node is one query over that node's F features
    MatchCall c;
    c.train = F;
    int KFit = 0, Fit = 0;
    while (KFit < n_kf_nodes && Fit < n_f_nodes) {
        if (kf_nodes[KFit] == f_nodes[Fit]) {
            for (int a = kf_ptr[KFit]; a < kf_ptr[KFit + 1]; a++) {
                const int idx = kf_feats[a];
                if (idx < 0 || idx >= kf->n) { set_error("KF feature index %d out of range", idx); return YGZFE_EINVAL; }
                ygzfe_match_query Q;
                memset(&Q, 0, sizeof(Q));
                Q.angle = kf->host_kps[idx].angle;
                Q.min_level = Q.max_level = -1;
                Q.flags = kf_usable[idx] ? YGZFE_MQ_VALID : 0;
                c.q.push_back(Q);
                c.qid.push_back(idx);
                c.cand_ptr.push_back(f_ptr[Fit]);
                c.cand_ptr.push_back(f_ptr[Fit + 1]);
            }
            KFit++;
            Fit++;
        } else if (kf_nodes[KFit] < f_nodes[Fit]) {
            KFit = (int)(std::lower_bound(kf_nodes + KFit, kf_nodes + n_kf_nodes, f_nodes[Fit]) - kf_nodes);
        } else {
            Fit = (int)(std::lower_bound(f_nodes + Fit, f_nodes + n_f_nodes, kf_nodes[KFit]) - f_nodes);
        }
    }
    const int n_cand = n_f_nodes > 0 ? f_ptr[n_f_nodes] : 0;
    for (int i = 0; i < n_cand; i++)
        if (f_feats[i] < 0 || f_feats[i] >= F->n) { set_error("F feature index %d out of range", f_feats[i]); return YGZFE_EINVAL; }
    c.cand_host = f_feats;
    c.n_cand = n_cand;
    if (c.cand_ptr.empty()) c.cand_ptr.assign(2, 0);  // BoW mode even with no query
    c.qdesc_dev = kf->desc.as<uint8_t>();
    c.qframe = kf;
    c.mode = YGZFE_MATCH_BOW;
    c.nnratio = nnratio;
    c.check_ori = check_ori;
    c.train_out = f_match;
    YGZ_TRY(run_match(c));
    *nmatches = c.nmatches;
    return YGZFE_OK;
}
