// rr_api.hip — C-ABI entry points (include/rain_raster.h): scratch carving, stage ordering,
// the single device->host sync, debug checks and event timing.
//
// Replaces CudaRasterizer::Rasterizer::{forward,backward,markVisible}
// (rasterizer_impl.cu:130-142,187-430) and the pybind wrappers (rasterize_points.cu:24-212).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rain_raster.h"
#include "rr_common.hpp"
#include "rr_kernels.hpp"

using namespace rr;

namespace rr {
// The tuning record of the current device (rr_kernels.hpp Tuning): a device index outside the
// table, or no device at all (a CPU-only process setting knobs), uses entry 0.
Tuning& tuning() {
    static Tuning per_device[kMaxDevices];
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDevices) {
        (void)hipGetLastError();
        d = 0;
    }
    return per_device[d];
}
}  // namespace rr

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// Bump allocator over an opaque byte buffer (rasterizer_impl.h:10-16 `obtain`).
struct Carver {
    char* base;
    size_t off = 0;
    explicit Carver(void* b) : base(static_cast<char*>(b)) {}
    template <typename T>
    T* take(size_t n) {
        off = align_up(off);
        T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
        off += n * sizeof(T);
        return p;
    }
};

// rasterizer_impl.cu:24-39
uint32_t higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

inline int grid_x(int W) { return (W + TILE_X - 1) / TILE_X; }
inline int grid_y(int H) { return (H + TILE_Y - 1) / TILE_Y; }


// ---- scratch layouts ----
struct Geom {
    Splat* splats;
    uint2* tiles;         // per Gaussian {pairs emitted, bounding-rect tiles}
    uint32_t* depth_keys;
    PhaseLists lists;     // the early-stop phases' Gaussians in index order with their pair offsets
    float4* normals;      // RR_FLAG_AUX_NORMAL: view-space normal per visible Gaussian
    uint2* block_sums;    // [ceil(P/256)] per-preprocess-block sums of tiles[] (pairs, rect tiles)
    uint32_t* block_wide; // [ceil(P/256)] per block: a visible depth key needs more than kDepthKeyBits
    FrameTotals* ft;      // the frame's counts and early-stop depth cut (rr_bin.hip)
    void* temp;           // the pair scan's block totals
    size_t temp_bytes;
    size_t total;
};
Geom carve_geom(void* buf, int P) {
    Carver c(buf);
    Geom g;
    const size_t n = (size_t)std::max(P, 1);
    g.splats = c.take<Splat>(n);
    g.tiles = c.take<uint2>(n);
    g.depth_keys = c.take<uint32_t>(n);
    g.lists.idx_a = c.take<uint32_t>(n);
    g.lists.off_a = c.take<uint32_t>(n);
    g.lists.idx_b = c.take<uint32_t>(n);
    g.lists.off_b = c.take<uint32_t>(n);
    // window starts for up to 2048 * P / 16 pairs per phase (more: a window-starts launch)
    g.lists.nwin = (uint32_t)std::min<size_t>(std::max<size_t>(n / 16, 64), (1u << 29) / kSplitWin + 1);
    g.lists.first_a = c.take<uint32_t>(g.lists.nwin);
    g.lists.first_b = c.take<uint32_t>(g.lists.nwin);
    g.normals = c.take<float4>(n);
    g.block_sums = c.take<uint2>((n + 255) / 256);
    g.block_wide = c.take<uint32_t>((n + 255) / 256);
    g.ft = c.take<FrameTotals>(1);
    g.temp_bytes = split_scan_temp_bytes(P);
    g.temp = c.take<char>(std::max<size_t>(g.temp_bytes, 1));
    g.total = align_up(c.off);
    return g;
}

struct Img {
    float* final_T;
    uint32_t* n_contrib;
    uint2* ranges;      // phase-A (or single-phase) lists; ranges_b and counters follow it
    uint2* ranges_b;    // phase-B lists of early-stop binning (all {0,0} otherwise)
    uint32_t* counters; // [0] phase-B pairs (gather path: slots reserved), [1] backward tile order done,
                        // [2] phase B took the gather path, [3] phase-B pairs its bin runs hold
    size_t zero_bytes;  // ranges .. bin_cnt_a: cleared before every render
    uint32_t* tile_max;
    uint8_t* open;      // [T] tile still open after phase A
    uint32_t* open_bits;  // [ceil(T/32)] open as a bitmask (in the zeroed block; the phase-A blend sets it)
    uint2* bounds_a;      // [bins] phase A's (or the single phase's) bin runs (zeroed block; k_bin_bounds)
    uint2* bounds_b;      // [bins] phase B's
    uint32_t* bin_cnt;    // [2 bins] phase B's pair count per bin (the gather path), then its fill
    uint32_t* bin_cnt_a;  // [2 bins] phase A's
    uint32_t* order;      // [T] backward blend dispatch order (heaviest tiles first)
    size_t total;
};
Img carve_img(void* buf, int W, int H) {
    Carver c(buf);
    Img m;
    const size_t N = (size_t)std::max(W * H, 1);
    const size_t T = (size_t)std::max(grid_x(W) * grid_y(H), 1);
    m.final_T = c.take<float>(N);
    m.n_contrib = c.take<uint32_t>(N);
    // one block, cleared before every render: ranges [T], ranges_b [T], counters [4],
    // open_bits [ceil(T/32)], bounds_a [bins], bounds_b [bins], bin_cnt [2 bins], bin_cnt_a [2 bins]
    const size_t nbits = ((size_t)T + 31) / 32;
    const size_t NB = (size_t)std::max(bins_x(grid_x(W)) * bins_y(grid_y(H)), 1);
    const size_t nz = 2 * (size_t)T + 2 + (nbits + 1) / 2 + 2 * NB + 2 * NB;
    m.ranges = c.take<uint2>(nz);
    m.ranges_b = m.ranges ? m.ranges + T : nullptr;
    m.counters = m.ranges ? reinterpret_cast<uint32_t*>(m.ranges + 2 * T) : nullptr;
    m.open_bits = m.ranges ? reinterpret_cast<uint32_t*>(m.ranges + 2 * T + 2) : nullptr;
    m.bounds_a = m.ranges ? m.ranges + 2 * T + 2 + (nbits + 1) / 2 : nullptr;
    m.bounds_b = m.ranges ? m.bounds_a + NB : nullptr;
    m.bin_cnt = m.ranges ? reinterpret_cast<uint32_t*>(m.bounds_b + NB) : nullptr;
    m.bin_cnt_a = m.ranges ? m.bin_cnt + 2 * NB : nullptr;
    m.zero_bytes = nz * sizeof(uint2);
    m.tile_max = c.take<uint32_t>(T);
    m.open = c.take<uint8_t>(T);
    m.order = c.take<uint32_t>(T);
    m.total = align_up(c.off);
    return m;
}

// Early-stop binning split (rr_bin.hip depth_cut): phase A bins the pairs of the Gaussians nearer
// than a per-frame depth cut holding ~1/den of the pairs, for every tile; phase B the rest, only for
// the tiles phase A left open (rr_kernels.hpp BlendPhase).  den = 3: on the bench frames (1M
// Gaussians, 1080p) most tiles saturate inside the first third (tools/saturation_stats.py; with the
// depth-rank split of rounds 1-3, tools/step_ab.py --split 2,3,4: 1.509 / 1.491 / 1.525 ms per
// step).  Frames below Tuning::early_min pairs are binned in one phase.  rr_set_binning_config
// changes both (tests force the split onto small frames).
//
// Binning paths: phase A (or the single phase) by the windowed duplicate over the split scan's
// index-ordered list + the stable bin sort; phase B by the gather path (rr_forward.hip k_dup_gather,
// per-bin count / scatter: few pairs) when the grid's bins fit one workgroup's count (rr_bin.hip
// kBinScanMax), else by the windowed path (Tuning::b_gather off forces it onto small frames).
constexpr int kGatherMaxBins = 16384;  // rr_bin.hip kBinScanMax
bool b_gather(int W, int H) {
    return tuning().b_gather && bins_x(grid_x(W)) * bins_y(grid_y(H)) <= kGatherMaxBins;
}

struct Bin {
    // FIRST, so the backward finds it without knowing the pair count: the per-tile lists
    // k_sortexpand writes, 4 slots per (bin, Gaussian) pair.  The host knows only the frame's
    // total L (the phases' split LA + LB = L stays on the device).  Every pair array has a phase-A
    // region [0, L) and a phase-B region [L, 2L) (point_list: [0, 4L) and [4L, 8L)), plus the bin
    // sort's arrays — 56 B per pair with 16-bit bin keys (point_list 32, keys 4 + 4 sorted, values
    // 8 + 8 sorted) + ~0.5 B of sort counts.
    // Bins of more than 2048 pairs are depth-sorted inside their own point_list region (rr_bin.hip
    // sortexpand_run): no scratch arrays.
    uint32_t* point_list;
    void* keys;            // bin ids of the (bin, Gaussian) pairs
    void* keys_sorted;
    uint32_t* vals;        // Gaussian | tile mask << BIN_SHIFT, then sorted
    uint32_t* vals_sorted;
    uint32_t* first;       // first Gaussian of every duplicate window (= sort unit), phase A then B
    uint32_t* unit_len;    // phase B: pairs kept per window
    void* temp;            // bin-sort scratch, shared by the two phases
    size_t temp_bytes;
    bool wide;  // 32-bit bin keys (more than 65536 bins)
    int bits;
    uint32_t L;  // (bin, Gaussian) pairs of both phases
    size_t total;
};
// Window (= sort unit) length of each phase's sort, chosen for the pairs it is expected to hold
// (the split scan's depth cut aims phase A at ~1/den of the pairs) while its windows cover the
// capacity L.
struct PhaseHints {
    size_t a, b;
};
PhaseHints phase_hints(uint32_t L, bool early) {
    const size_t n = std::max<size_t>(L, 1);
    const size_t a = std::max<size_t>(n / std::max<uint32_t>(tuning().early_den, 1u), 1);
    return early ? PhaseHints{a, std::max<size_t>(n - a, 1)} : PhaseHints{n, n};
}
template <typename K>
RadixPlan tile_plan(void* temp, uint32_t n, int bits, size_t hint) {
    return radix_sort_plan<K>(temp, (size_t)n, 0, bits, hint);
}
// The layout depends on the frame's pair count L only, sized for the early-stop split (its
// phase-A hint has the most windows; a single-phase frame uses fewer).
Bin carve_bin(void* buf, int L, int W, int H) {
    Carver c(buf);
    Bin b;
    const int NB = bins_x(grid_x(W)) * bins_y(grid_y(H));
    b.wide = NB > 65536 || tuning().wide_bin_keys;
    b.bits = std::max(1, (int)higher_msb((uint32_t)NB));  // >= 1: the duplicate windows are sort units
    b.L = (uint32_t)std::max(L, 0);
    const size_t np = 2 * (size_t)std::max(L, 1);  // entries of each pair array: both phases' regions
    b.point_list = c.take<uint32_t>(4 * np + kPointListPad);
    if (b.wide) {
        b.keys = c.take<uint32_t>(np);
        b.keys_sorted = c.take<uint32_t>(np);
    } else {
        b.keys = c.take<uint16_t>(np);
        b.keys_sorted = c.take<uint16_t>(np);
    }
    b.vals = c.take<uint32_t>(np);
    b.vals_sorted = c.take<uint32_t>(np);
    {
        const PhaseHints h = phase_hints(b.L, true);
        auto units = [&](size_t hint) {
            return b.wide ? tile_plan<uint32_t>(nullptr, b.L, b.bits, hint).units
                          : tile_plan<uint16_t>(nullptr, b.L, b.bits, hint).units;
        };
        const int ua = std::max(units(h.a), 1), ub = std::max(units(h.b), 1);
        b.first = c.take<uint32_t>((size_t)ua + ub + 2);
        b.unit_len = c.take<uint32_t>((size_t)ub + 1);
        auto temp = [&](size_t hint) {
            return b.L == 0 ? (size_t)0
                   : b.wide ? radix_sort_temp_bytes<uint32_t>(b.L, b.bits, hint)
                            : radix_sort_temp_bytes<uint16_t>(b.L, b.bits, hint);
        };
        b.temp_bytes = std::max(temp(h.a), temp(h.b));
        b.temp = c.take<char>(std::max<size_t>(b.temp_bytes, 1));
    }
    b.total = align_up(c.off);
    return b;
}

// ---- event timing (bench.py reads per-stage kernel time through rr_profile_collect) ----
struct EvRec {
    int stage;
    hipEvent_t a, b;
};
bool g_prof = false;
unsigned g_prof_mask = 0xffffffffu;  // stages recorded while profiling (rr_profile_select)
std::vector<EvRec> g_recs;
std::vector<hipEvent_t> g_pool;

hipEvent_t ev_get() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    // timing only: no system-scope fence (cache write-back + invalidate) at each record, which
    // otherwise opens a ~5 us gap before the next kernel of the stream
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipEventCreate(&e);
    }
    return e;
}

struct StageTimer {
    int stage;
    hipStream_t st;
    hipEvent_t a = nullptr;
    StageTimer(int s, hipStream_t stream) : stage(s), st(stream) {
        if (g_prof && ((g_prof_mask >> s) & 1u)) {
            a = ev_get();
            (void)hipEventRecord(a, st);
        }
    }
    ~StageTimer() {
        if (a) {
            hipEvent_t b = ev_get();
            (void)hipEventRecord(b, st);
            g_recs.push_back({stage, a, b});
        }
    }
};

// Launch check: always catch launch errors; with `debug`, synchronise and check the kernel
// (CHECK_CUDA, auxiliary.h:155-162).
int check(const rr_frame* f, hipStream_t st, const char* what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && f && f->debug) {
        e = hipStreamSynchronize(st);
        if (e == hipSuccess) e = hipGetLastError();
    }
    if (e != hipSuccess) return fail(RR_ERR_HIP, std::string("[HIP ERROR] in ") + what + ": " + hipGetErrorString(e));
    return RR_OK;
}
#define RR_CHECK(call, what)                                                              \
    do {                                                                                  \
        hipError_t _e = (call);                                                           \
        if (_e != hipSuccess)                                                             \
            return fail(RR_ERR_HIP, std::string("[HIP ERROR] ") + what + ": " + hipGetErrorString(_e)); \
    } while (0)
#define RR_STAGE_CHECK(what)                   \
    do {                                       \
        int _rc = check(f, st, what);          \
        if (_rc != RR_OK) return _rc;          \
    } while (0)

// ---------------------------------------------------------------------------------------
// Readback of the forward's pair counts.  A hipMemcpyAsync into pageable host memory + stream
// synchronise after the scan costs a blit kernel and the runtime's blocking wait (measured 30-140
// us of idle GPU per frame before the binning launches).  Instead the split scan's first launch
// (rr_bin.hip k_split_scan_totals: workgroup 0, once the frame's totals and depth cut are known;
// the scan runs on while the host reads) stores the counts and a sequence number into a coherent
// pinned host mailbox (system-scope stores, the sequence number last) and the host thread spins on
// the sequence number.  Once the
// wait has outlasted any frame the stream is queried: a launch / kernel error is reported, and a
// stream that went idle without the sequence number becoming visible falls back to the plain copy.
struct Mailbox {
    uint32_t* host = nullptr;  // [L, rect, seq, wide], coherent pinned
    uint32_t* dev = nullptr;   // device alias of host
    uint32_t seq = 0;
    bool failed = false;       // allocation failed: always use the copy
};
thread_local Mailbox g_mailbox;

struct PairCountRead {
    const FrameTotals* copy = nullptr;  // device totals for the copy path
    uint32_t seq = 0;  // 0: no mailbox (copy + synchronise at wait time)
};
struct PairCounts {
    uint32_t L = 0, rect = 0;  // saturated to 32 bits
    bool wide = false;
};

// The mailbox (allocated on first use) and this read's sequence number; box == null: no mailbox.
uint32_t* pair_counts_box(const FrameTotals* copy, PairCountRead& r) {
    Mailbox& mb = g_mailbox;
    r.copy = copy;
    r.seq = 0;
    if (!mb.host && !mb.failed) {
        void* h = nullptr;
        if (hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
            hipHostGetDevicePointer(reinterpret_cast<void**>(&mb.dev), h, 0) == hipSuccess) {
            mb.host = static_cast<uint32_t*>(h);
            std::memset(h, 0, 64);
        } else {
            if (h) (void)hipHostFree(h);
            (void)hipGetLastError();
            mb.failed = true;
        }
    }
    if (mb.failed) return nullptr;
    r.seq = ++mb.seq == 0 ? ++mb.seq : mb.seq;  // 0 is the mailbox's initial value
    return mb.dev;
}

hipError_t pair_counts_copy(const FrameTotals* src, PairCounts* out, hipStream_t st) {
    FrameTotals v{};
    hipError_t e = hipMemcpyAsync(&v, src, sizeof(v), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    out->L = v.L > 0xffffffffull ? 0xffffffffu : (uint32_t)v.L;
    out->rect = v.rect > 0xffffffffull ? 0xffffffffu : (uint32_t)v.rect;
    out->wide = v.wide != 0;
    return e;
}

thread_local int64_t g_wait_ns = 0, g_waits = 0;
#ifndef RR_WAIT_QUERY_MS
#define RR_WAIT_QUERY_MS 20
#endif
struct WaitClock {  // adds the scope's duration to the host-wait statistics
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~WaitClock() {
        g_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        g_waits++;
    }
};

hipError_t pair_counts_wait(const PairCountRead& r, PairCounts* out, hipStream_t st) {
    WaitClock clock;
    Mailbox& mb = g_mailbox;
    if (r.seq == 0) return pair_counts_copy(r.copy, out, st);
    for (uint32_t spin = 1;; spin++) {
        if (__atomic_load_n(mb.host + 2, __ATOMIC_ACQUIRE) == r.seq) {
            out->L = __atomic_load_n(mb.host + 0, __ATOMIC_RELAXED);
            out->rect = __atomic_load_n(mb.host + 1, __ATOMIC_RELAXED);
            out->wide = __atomic_load_n(mb.host + 3, __ATOMIC_RELAXED) != 0;
            return hipSuccess;
        }
        // the stream is queried only once the wait has outlasted any frame (RR_WAIT_QUERY_MS): a query
        // while the device is still busy with this frame is not free on the device side
        if ((spin & 4095u) == 0 &&
            std::chrono::steady_clock::now() - clock.t0 > std::chrono::milliseconds(RR_WAIT_QUERY_MS)) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) {
                if (__atomic_load_n(mb.host + 2, __ATOMIC_ACQUIRE) == r.seq) continue;
                mb.failed = true;  // idle stream, value not visible: never use the mailbox again
                return pair_counts_copy(r.copy, out, st);
            }
            if (q != hipErrorNotReady) return q;
        }
        __builtin_ia32_pause();
    }
}

int validate(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, bool forward) {
    if (!f || !cam || !g) return fail(RR_ERR_ARG, "null frame/camera/gaussians");
    if (f->P < 0 || f->width <= 0 || f->height <= 0) return fail(RR_ERR_ARG, "bad P/width/height");
    if (f->P > (int)BIN_ID_MASK) return fail(RR_ERR_ARG, "P >= 2^28 (pair values carry a 4-bit tile mask)");
    if (f->P == 0) return RR_OK;
    if (!g->means3D || (forward && !g->opacities)) return fail(RR_ERR_ARG, "means3D and opacities are required");
    if (!cam->background || !cam->viewmatrix || !cam->projmatrix || !cam->campos)
        return fail(RR_ERR_ARG, "camera arrays are required");
    if ((g->shs == nullptr) == (g->colors_precomp == nullptr))
        return fail(RR_ERR_ARG, "Please provide excatly one of either SHs or precomputed colors!");
    const bool sr = g->scales && g->rotations;
    if (sr == (g->cov3D_precomp != nullptr))
        return fail(RR_ERR_ARG,
                    "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    if (g->shs && (f->D < 0 || f->D > 3 || f->M < (f->D + 1) * (f->D + 1)))
        return fail(RR_ERR_ARG, "sh_degree must be 0..3 and sh.size(1) >= (degree+1)^2");
    if (f->M > 16) return fail(RR_ERR_ARG, "sh.size(1) > 16 is not supported (SH degree <= 3, forward.cu:9-60)");
    if ((f->flags & RR_FLAG_AUX_NORMAL) && !sr)
        return fail(RR_ERR_ARG, "the aux normal output needs scales/rotations (not cov3D_precomp)");
    if (f->flags & RR_FLAG_RAW_PARAMS) {
        if (!g->shs || !sr || !g->opacities)
            return fail(RR_ERR_ARG, "raw-parameter mode needs SH, scales/rotations and opacities");
        if (f->M > 1 && !g->shs_rest) return fail(RR_ERR_ARG, "raw-parameter mode needs shs_rest when M > 1");
    }
    return RR_OK;
}

// Preprocess arguments of a frame (the output arrays are set by the caller).
PreArgs pre_args(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g) {
    PreArgs a{};
    a.P = f->P; a.D = f->D; a.M = f->M; a.W = f->width; a.H = f->height;
    a.gx = grid_x(f->width); a.gy = grid_y(f->height);
    a.prefiltered = f->prefiltered;
    a.tanfovx = f->tan_fovx; a.tanfovy = f->tan_fovy;
    a.focal_y = f->height / (2.0f * f->tan_fovy);
    a.focal_x = f->width / (2.0f * f->tan_fovx);
    a.scale_modifier = f->scale_modifier; a.low_pass = f->low_pass;
    a.means3D = g->means3D; a.shs = g->shs; a.colors_precomp = g->colors_precomp; a.opacities = g->opacities;
    a.scales = g->scales; a.rotations = g->rotations; a.cov3D_precomp = g->cov3D_precomp;
    a.view = cam->viewmatrix; a.proj = cam->projmatrix; a.campos = cam->campos;
    a.cull = (f->flags & RR_FLAG_NO_TILE_CULLING) ? 0 : 1;
    a.raw = (f->flags & RR_FLAG_RAW_PARAMS) ? 1 : 0;
    a.shs_rest = g->shs_rest;
    return a;
}

// The image buffer whose per-frame block the last pair count of this thread cleared, not yet
// rendered into: a render consumes it, so that a second render after one pair count (whose gather
// counters would start where the first one's ended, past their regions) fails instead.
thread_local const void* g_counted_img = nullptr;

// Depth cut + the split pair-count scan -> the one device->host read of the forward, over a
// geometry buffer whose per-Gaussian arrays (splats, tiles, depth keys, block sums) are filled.  No
// depth sort: the bins' runs are put in depth order by k_sortexpand (rr_bin.hip).  The scan's first
// launch computes the cut and clears the image buffer's per-frame block (im: the buffer the frame
// is then rendered into).
int count_pairs(const rr_frame* f, const Geom& gm, const Img& im, int P, hipStream_t st, int* num_rendered,
                int* num_pairs) {
    PairCountRead rd;
    uint32_t* box = pair_counts_box(gm.ft, rd);
    const bool full = (f->flags & RR_FLAG_FULL_BINNING) != 0;
    const Tuning& tu = tuning();
    {
        StageTimer tm(RR_STAGE_SCAN, st);
        uint32_t* zero = reinterpret_cast<uint32_t*>(im.ranges);
        const int nzero = (int)(im.zero_bytes / sizeof(uint32_t));
        const CutArgs ca{gm.block_sums, gm.block_wide, full ? 1u : tu.early_den, tu.early_min, box, rd.seq};
        launch_split_scan(gm.tiles, gm.depth_keys, P, gm.lists, gm.ft, gm.temp, tu.pair_scan_direct_blocks, zero,
                          nzero, ca, st);
        RR_CHECK(hipGetLastError(), "pair-count scan");
    }
    g_counted_img = im.final_T;
    RR_STAGE_CHECK("scan");
    // the one device->host sync of the forward (rasterizer_impl.cu:273): pairs to bin, and the
    // reference's num_rendered (sum of bounding-rect areas) which the API returns unchanged; the
    // split into the early-stop phases stays on the device
    PairCounts c;
    RR_CHECK(pair_counts_wait(rd, &c, st), "read L");
    if (c.L > 0x1fffffffu || c.rect > 0x7fffffffu) return fail(RR_ERR_CAPACITY, "more than 2^29 bin/Gaussian pairs");
    *num_rendered = (int)c.rect;
    *num_pairs = (int)c.L;
    return RR_OK;
}

}  // namespace

extern "C" {

const char* rr_last_error(void) { return g_err.c_str(); }
const char* rr_version(void) { return "rain_amd-raster 0.1 gfx950"; }

size_t rr_geometry_bytes(int P) { return carve_geom(nullptr, P).total; }
size_t rr_image_bytes(int width, int height) { return carve_img(nullptr, width, height).total; }
size_t rr_binning_bytes(int num_rendered, int width, int height) {
    return carve_bin(nullptr, num_rendered, width, height).total;
}
size_t rr_backward_workspace_bytes(int P) { return align_up((size_t)std::max(P, 1) * GACC_STRIDE * sizeof(float)); }

int rr_forward_geometry(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, int* radii, void* geom_buffer,
                        size_t geom_bytes, void* image_buffer, size_t image_bytes, int* num_rendered,
                        int* num_pairs, void* stream) {
    int rc = validate(f, cam, g, true);
    if (rc) return rc;
    if (!num_rendered || !num_pairs) return fail(RR_ERR_ARG, "num_rendered / num_pairs is null");
    *num_rendered = 0;
    *num_pairs = 0;
    const int P = f->P, W = f->width, H = f->height;
    if (P == 0) return RR_OK;
    if (!radii || !geom_buffer || !image_buffer) return fail(RR_ERR_ARG, "null output buffer");
    const Geom gm = carve_geom(geom_buffer, P);
    const Img im = carve_img(image_buffer, W, H);
    if (geom_bytes < gm.total || image_bytes < im.total) return fail(RR_ERR_CAPACITY, "scratch buffer too small");
    hipStream_t st = (hipStream_t)stream;
    PreArgs a = pre_args(f, cam, g);
    a.radii = radii; a.splats = gm.splats; a.tiles = gm.tiles; a.depth_keys = gm.depth_keys;
    a.normals = (f->flags & RR_FLAG_AUX_NORMAL) ? gm.normals : nullptr;
    a.block_sums = gm.block_sums;
    a.block_wide = gm.block_wide;
    {
        StageTimer tm(RR_STAGE_PREPROCESS, st);
        launch_preprocess(a, st);
    }
    RR_STAGE_CHECK("preprocess");
    return count_pairs(f, gm, im, P, st, num_rendered, num_pairs);
}

}  // extern "C"

namespace {

// The backward's accumulator workspace: registered for the next forward render on this thread
// (rr_set_forward_workspace), which zero-fills it inside its first blend launch.
struct WsRange {
    void* ptr = nullptr;
    size_t bytes = 0;
};
thread_local WsRange g_fwd_ws;
// What a render leaves for its frame's backward, which may run on another host thread (autograd's
// device thread): the workspace it zero-filled, and the backward's tile order when its phase-B
// duplicate launch computed it (the order array).  A backward whose workspace is the clean one
// skips its clear, and with the order ready it needs no prologue at all.  Process-wide, keyed by
// the image buffer, the last few renders; the first backward of a frame consumes its entry (a
// second one, of a retained graph, clears and orders by itself).
struct FrameFacts {
    const void* img = nullptr;
    WsRange clean;
    const uint32_t* order = nullptr;
};
std::mutex g_facts_mu;
std::deque<FrameFacts> g_facts;
constexpr size_t kMaxFacts = 16;
thread_local FrameFacts g_render_facts;  // the facts of the render in progress on this thread
void publish_facts(const FrameFacts& f) {
    std::lock_guard<std::mutex> lk(g_facts_mu);
    for (auto it = g_facts.begin(); it != g_facts.end(); ++it)
        if (it->img == f.img) {
            g_facts.erase(it);
            break;
        }
    if (f.clean.ptr || f.order) g_facts.push_back(f);
    if (g_facts.size() > kMaxFacts) g_facts.pop_front();
}
FrameFacts take_facts(const void* img) {
    std::lock_guard<std::mutex> lk(g_facts_mu);
    for (auto it = g_facts.begin(); it != g_facts.end(); ++it)
        if (it->img == img) {
            const FrameFacts f = *it;
            g_facts.erase(it);
            return f;
        }
    return FrameFacts{};
}

// Tile lists for one frame: duplicate -> pairs into their bins -> per-bin depth order + tile lists
// -> blend, once (single phase) or as the two phases of early-stop binning (rr_kernels.hpp
// BlendPhase).  The host knows the frame's total L only: phase A's pairs go to region [0, L) of the
// pair arrays and phase B's to region [L, 2L); every launch is sized for L and reads its phase's
// count on the device (FrameTotals LA / LB, or the gather path's counters).
template <typename K>
int render_tiles(const rr_frame* f, const Geom& gm, const Img& im, const Bin& bn, const int* radii, int P, int W,
                 int H, int cull, bool early, BlendFwdArgs b, hipStream_t st) {
    const int gx = grid_x(W), gy = grid_y(H);
    const uint32_t L = bn.L;
    K* keys = static_cast<K*>(bn.keys);
    K* keys_sorted = static_cast<K*>(bn.keys_sorted);
    DupArgs<K> d{};
    d.P = P; d.splats = gm.splats; d.radii = radii;
    d.gx = gx; d.gy = gy; d.cull = cull;
    d.tiles = gm.tiles;
    const PhaseHints h = phase_hints(L, early);
    const bool gather = early && b_gather(W, H);
    const RadixPlan pa = tile_plan<K>(bn.temp, L, bn.bits, h.a);  // phase A (or the only phase)
    const RadixPlan pb = tile_plan<K>(bn.temp, L, bn.bits, h.b);  // phase B (windowed path)
    bool starts_b = false;  // phase B's window starts computed with phase A's
    // window starts marked by the split scan (units of kSplitWin pairs), else a window-starts launch
    const bool marks_a = pa.unit_items == kSplitWin && (uint32_t)pa.units <= gm.lists.nwin;
    const bool marks_b = pb.unit_items == kSplitWin && (uint32_t)pb.units <= gm.lists.nwin;
    // phase A (or the only phase): its pairs for every tile
    {
        StageTimer tm(RR_STAGE_DUPLICATE, st);
        d.n_list = &gm.ft->GA; d.idx = gm.lists.idx_a; d.off = gm.lists.off_a;
        d.first = marks_a ? gm.lists.first_a : bn.first;
        d.pair0 = 0; d.win = (uint32_t)pa.unit_items; d.nwin = pa.units; d.L_dev = &gm.ft->LA;
        d.keys = keys; d.vals = bn.vals; d.dbits = pa.dbits0; d.counts = pa.counts;
        d.starts_done = marks_a;
        if (early && !gather && !marks_a && !marks_b) {
            d.first_b = bn.first + pa.units; d.pair0_b = 0; d.win_b = (uint32_t)pb.unit_items; d.nwin_b = pb.units;
            d.n_list_b = &gm.ft->GB; d.off_b = gm.lists.off_b;
        }
        starts_b = launch_duplicate<K>(d, st);
        d.first_b = nullptr; d.nwin_b = 0; d.starts_done = false;
    }
    RR_STAGE_CHECK("duplicate");
    {
        StageTimer tm(RR_STAGE_TILE_SORT, st);
        RR_CHECK(radix_sort_pairs<K>(bn.temp, bn.temp_bytes, keys, keys_sorted, bn.vals, bn.vals_sorted, L, 0, bn.bits,
                                     st, true, nullptr, &gm.ft->LA, h.a, im.bounds_a),
                 std::string("bin sort (") + radix_sort_last_error() + ")");
    }
    RR_STAGE_CHECK("bin sort");
    {
        StageTimer tm(RR_STAGE_RANGES, st);
        launch_sortexpand<K>(keys_sorted, bn.vals_sorted, gm.depth_keys, gm.ft, gx, gy, 0u, bn.point_list, im.ranges,
                             nullptr, im.bounds_a, st);
    }
    RR_STAGE_CHECK("sort-expand");
    {
        StageTimer tm(RR_STAGE_BLEND_FWD, st);
        b.phase = early ? kBlendPhaseA : kBlendSingle;
        // the registered backward workspace (render_frame), cleared in this launch's drain
        if (b.clear) g_render_facts.clean = WsRange{b.clear, b.clear_n4 * sizeof(float4)};
        launch_blend_fwd(b, st);
        b.clear = nullptr;
        b.clear_n4 = 0;
    }
    RR_STAGE_CHECK("blend forward");
    if (!early) return RR_OK;
    // phase B: its pairs, only for tiles phase A left open; region [L, 2L) of the pair arrays.  The
    // backward's tile order is computed on phase A's tile_max by an extra workgroup of the phase-B
    // duplicate launch (counters[1] = T marks it done)
    d.open_bits = im.open_bits; d.n_total = im.counters;
    d.order_cost = im.tile_max; d.order_out = im.order; d.order_flag = im.counters + 1; d.order_T = gx * gy;
    if (gather) {
        {
            StageTimer tm(RR_STAGE_DUPLICATE, st);
            d.keys = keys + L; d.vals = bn.vals + L;
            d.n_list = &gm.ft->GB; d.idx = gm.lists.idx_b;
            d.gather_mark = im.counters + 2;
            if (P > 0) g_render_facts.order = im.order;
            launch_dup_gather<K>(d, st);
        }
        RR_STAGE_CHECK("duplicate (phase B gather)");
        {
            StageTimer tm(RR_STAGE_RANGES, st);
            // phase B's tile lists right after phase A's
            launch_sortexpand_small<K>(P, keys + L, bn.vals + L, im.counters, im.bin_cnt, bn.vals_sorted + L,
                                       gm.depth_keys, gm.ft, gx, gy, 4u * L, bn.point_list, im.ranges_b, im.open_bits,
                                       im.bounds_b, im.counters + 3, st);
        }
        RR_STAGE_CHECK("sort-expand (phase B gather)");
    } else {
        {
            StageTimer tm(RR_STAGE_DUPLICATE, st);
            d.n_list = &gm.ft->GB; d.idx = gm.lists.idx_b; d.off = gm.lists.off_b;
            d.first = marks_b ? gm.lists.first_b : bn.first + pa.units;
            d.pair0 = 0; d.win = (uint32_t)pb.unit_items; d.nwin = pb.units;
            d.L_dev = &gm.ft->LB;
            d.keys = keys + L; d.vals = bn.vals + L; d.dbits = pb.dbits0; d.counts = pb.counts;
            d.unit_len = bn.unit_len;
            d.zero = nullptr; d.nzero = 0;
            d.starts_done = starts_b || marks_b;
            if (P > 0) g_render_facts.order = im.order;
            launch_duplicate<K>(d, st);
        }
        RR_STAGE_CHECK("duplicate (phase B)");
        {
            StageTimer tm(RR_STAGE_TILE_SORT, st);
            RR_CHECK(radix_sort_pairs<K>(bn.temp, bn.temp_bytes, keys + L, keys_sorted + L, bn.vals + L,
                                         bn.vals_sorted + L, L, 0, bn.bits, st, true, bn.unit_len, im.counters, h.b,
                                         im.bounds_b),
                     std::string("bin sort, phase B (") + radix_sort_last_error() + ")");
        }
        RR_STAGE_CHECK("bin sort (phase B)");
        {
            StageTimer tm(RR_STAGE_RANGES, st);
            launch_sortexpand<K>(keys_sorted + L, bn.vals_sorted + L, gm.depth_keys, gm.ft, gx, gy, 4u * L,
                                 bn.point_list, im.ranges_b, im.open_bits, im.bounds_b, st);
        }
        RR_STAGE_CHECK("sort-expand (phase B)");
    }
    {
        StageTimer tm(RR_STAGE_BLEND_FWD, st);
        b.phase = kBlendPhaseB;
        launch_blend_fwd(b, st);
    }
    RR_STAGE_CHECK("blend forward (phase B)");
    return RR_OK;
}

int render_frame(const rr_frame* f, const rr_camera* cam, const int* radii, void* geom_buffer, void* image_buffer,
                 void* binning_buffer, size_t binning_bytes, int num_pairs, float* out_color, float* out_depth,
                 float* out_normal, void* stream);int render_frame(const rr_frame* f, const rr_camera* cam, const int* radii, void* geom_buffer, void* image_buffer,
                 void* binning_buffer, size_t binning_bytes, int num_pairs, float* out_color, float* out_depth,
                 float* out_normal, void* stream);

// Accumulator clear (+ the backward's tile order) and the blend backward: gacc [P][GACC_STRIDE]
// receives every Gaussian's dmean2D / dconic / dopacity / dcolor sums of the frame.
int blend_backward(const rr_frame* f, const rr_camera* cam, const void* geom_buffer, const void* image_buffer,
                   const void* binning_buffer, int L, const float* dL_dpix, float* gacc, hipStream_t st) {
    const int P = f->P, W = f->width, H = f->height;
    const Geom gm = carve_geom(const_cast<void*>(geom_buffer), P);
    const Img im = carve_img(const_cast<void*>(image_buffer), W, H);
    // point_list sits at the start of the binning buffer, so its position does not depend on the
    // pair count; tiles whose forward blended nothing (tile_max 0) never read it
    const Bin bn = carve_bin(const_cast<void*>(binning_buffer), 0, W, H);
    const int gx = grid_x(W), gy = grid_y(H);
    const bool blend = L > 0 && binning_buffer;
    uint32_t* order = blend ? im.order : nullptr;  // heaviest tiles first
    // the accumulators already zero-filled by the forward (rr_set_forward_workspace): no clear
    const size_t nacc = (size_t)P * GACC_STRIDE;
    const FrameFacts facts = take_facts(im.final_T);  // this backward's accumulation dirties the workspace
    const bool clean = (f->flags & RR_FLAG_WORKSPACE_REGISTERED) && facts.clean.ptr == gacc &&
                       facts.clean.bytes >= nacc * sizeof(float);
    const bool order_ready = order && facts.order == order;
    if (!clean || (order && !order_ready)) {
        StageTimer tm(RR_STAGE_MEMSET, st);
        launch_bwd_prologue(gacc, clean ? 0 : nacc, gx * gy, im.tile_max, order_ready ? nullptr : order,
                            im.counters + 1, st);
        RR_CHECK(hipGetLastError(), "clear accumulators");
    }
    if (blend) {
        StageTimer tm(RR_STAGE_BLEND_BWD, st);
        BlendBwdArgs b{};
        b.W = W; b.H = H; b.gx = gx; b.gy = gy;
        b.ranges = im.ranges; b.ranges_b = im.ranges_b; b.point_list = bn.point_list; b.splats = gm.splats;
        b.tile_max = im.tile_max;
        b.final_T = im.final_T; b.n_contrib = im.n_contrib; b.bg = cam->background; b.dL_dpix = dL_dpix;
        b.gacc = gacc;
        b.order = order;
        launch_blend_bwd(b, st);
    }
    RR_STAGE_CHECK("blend backward");
    return RR_OK;
}

}  // namespace

extern "C" {

int rr_forward_render(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, const int* radii,
                      void* geom_buffer, void* image_buffer, void* binning_buffer, size_t binning_bytes,
                      int num_pairs, float* out_color, float* out_depth, void* stream) {
    if (f && (f->flags & RR_FLAG_AUX_NORMAL)) return fail(RR_ERR_ARG, "RR_FLAG_AUX_NORMAL: use rr_forward_render_aux");
    return rr_forward_render_aux(f, cam, g, radii, geom_buffer, image_buffer, binning_buffer, binning_bytes, num_pairs,
                                 out_color, out_depth, nullptr, stream);
}

int rr_forward_render_aux(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, const int* radii,
                          void* geom_buffer, void* image_buffer, void* binning_buffer, size_t binning_bytes,
                          int num_pairs, float* out_color, float* out_depth, float* out_normal, void* stream) {
    int rc = validate(f, cam, g, true);
    if (rc) return rc;
    if (((f->flags & RR_FLAG_AUX_NORMAL) != 0) != (out_normal != nullptr))
        return fail(RR_ERR_ARG, "out_normal must be given exactly when RR_FLAG_AUX_NORMAL is set");
    return render_frame(f, cam, radii, geom_buffer, image_buffer, binning_buffer, binning_bytes, num_pairs, out_color,
                        out_depth, out_normal, stream);
}

}  // extern "C"

namespace {

// Binning + blend of a frame whose pairs were just counted (count_pairs) into this image buffer.
int render_frame(const rr_frame* f, const rr_camera* cam, const int* radii, void* geom_buffer, void* image_buffer,
                 void* binning_buffer, size_t binning_bytes, int num_pairs, float* out_color, float* out_depth,
                 float* out_normal, void* stream) {
    const int P = f->P, W = f->width, H = f->height, L = num_pairs;
    const int cull = (f->flags & RR_FLAG_NO_TILE_CULLING) ? 0 : 1;
    // a workspace registration is used by this render (or dropped by it) either way
    const WsRange reg = g_fwd_ws;
    g_fwd_ws = WsRange{};
    if (P == 0) return RR_OK;
    if (!out_color || !out_depth || !geom_buffer || !image_buffer || (L > 0 && !binning_buffer))
        return fail(RR_ERR_ARG, "null buffer");
    const Geom gm = carve_geom(geom_buffer, P);
    const Img im = carve_img(image_buffer, W, H);
    if (g_counted_img != im.final_T)
        return fail(RR_ERR_ARG, "render without a pair count of this image buffer (one render per rr_forward_geometry / "
                                "rr_forward_from_geometry on this thread)");
    g_counted_img = nullptr;
    g_render_facts = FrameFacts{im.final_T, WsRange{}, nullptr};
    publish_facts(g_render_facts);  // drops an earlier render's facts of this buffer
    const Bin bn = carve_bin(binning_buffer, L, W, H);
    if (L > 0 && binning_bytes < bn.total) return fail(RR_ERR_CAPACITY, "binning buffer too small");
    hipStream_t st = (hipStream_t)stream;
    const int gx = grid_x(W), gy = grid_y(H);
    // (the per-frame block of the image buffer was cleared by count_pairs' split scan)
    BlendFwdArgs b{};
    b.W = W; b.H = H; b.gx = gx; b.gy = gy;
    b.ranges = im.ranges; b.ranges_b = im.ranges_b; b.open = im.open; b.open_bits = im.open_bits;
    b.point_list = bn.point_list; b.splats = gm.splats; b.bg = cam->background;
    b.final_T = im.final_T; b.n_contrib = im.n_contrib; b.tile_max = im.tile_max;
    b.clear = static_cast<float4*>(reg.ptr);
    b.clear_n4 = reg.bytes / sizeof(float4);
    b.out_color = out_color; b.out_depth = out_depth;
    b.normals = out_normal ? gm.normals : nullptr; b.out_normal = out_normal;
    if (L == 0) {  // no pairs: every tile keeps the background (one blend over empty lists)
        StageTimer tm(RR_STAGE_BLEND_FWD, st);
        b.phase = kBlendSingle;
        launch_blend_fwd(b, st);
        if (b.clear) g_render_facts.clean = WsRange{b.clear, b.clear_n4 * sizeof(float4)};
        const int rc = check(f, st, "blend forward");
        if (rc == RR_OK) publish_facts(g_render_facts);
        return rc;
    }
    // the split the depth cut makes (its one-phase conditions but "no sampled pair", which leaves
    // phase B empty on the device)
    const Tuning& tu = tuning();
    const bool early = !(f->flags & RR_FLAG_FULL_BINNING) && tu.early_den > 1 && (uint32_t)L >= tu.early_min;
    const int rc = bn.wide ? render_tiles<uint32_t>(f, gm, im, bn, radii, P, W, H, cull, early, b, st)
                           : render_tiles<uint16_t>(f, gm, im, bn, radii, P, W, H, cull, early, b, st);
    if (rc == RR_OK) publish_facts(g_render_facts);
    return rc;
}

}  // namespace

extern "C" {

int rr_forward(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, int* radii, void* geom_buffer,
               size_t geom_bytes, void* image_buffer, size_t image_bytes, void* binning_buffer, size_t binning_bytes,
               int* num_rendered, int* num_pairs, size_t* binning_needed, float* out_color, float* out_depth,
               void* stream) {
    if (!binning_needed) return fail(RR_ERR_ARG, "binning_needed is null");
    *binning_needed = 0;
    int rc = rr_forward_geometry(f, cam, g, radii, geom_buffer, geom_bytes, image_buffer, image_bytes, num_rendered,
                                 num_pairs, stream);
    if (rc != RR_OK || f->P == 0) return rc;
    const size_t need = *num_pairs > 0 ? carve_bin(nullptr, *num_pairs, f->width, f->height).total : 0;
    *binning_needed = need;
    if (binning_bytes < need) return RR_INCOMPLETE;
    return rr_forward_render(f, cam, g, radii, geom_buffer, image_buffer, binning_buffer, binning_bytes, *num_pairs,
                             out_color, out_depth, stream);
}

int rr_backward(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, const int* radii,
                const void* geom_buffer, const void* image_buffer, const void* binning_buffer, int num_rendered,
                const float* dL_dpix, void* workspace, size_t workspace_bytes, const rr_grads* out, void* stream) {
    int rc = validate(f, cam, g, false);
    if (rc) return rc;
    const int P = f->P, W = f->width, H = f->height, L = num_rendered;
    if (P == 0) return RR_OK;
    if (!out || !dL_dpix || !radii || !geom_buffer || !image_buffer || !workspace)
        return fail(RR_ERR_ARG, "null buffer");
    const bool raw = (f->flags & RR_FLAG_RAW_PARAMS) != 0;
    const rr_adam* ad = out->adam;
    if (ad && !raw) return fail(RR_ERR_ARG, "the fused optimizer step needs raw-parameter mode");
    if (ad) {
        const rr_adam_group* gs[6] = {&ad->xyz, &ad->f_dc, &ad->f_rest, &ad->opacity, &ad->scaling, &ad->rotation};
        const void* in[6] = {g->means3D, g->shs, g->shs_rest, g->opacities, g->scales, g->rotations};
        for (int i = 0; i < 6; i++) {
            if (i == 2 && f->M <= 1) continue;
            if (!gs[i]->param || !gs[i]->exp_avg || !gs[i]->exp_avg_sq)
                return fail(RR_ERR_ARG, "null Adam group array");
            if (gs[i]->param != in[i]) return fail(RR_ERR_ARG, "Adam group param must be the matching input array");
        }
    } else if (!out->dL_dopacity || !out->dL_dmeans3D || !out->dL_dscales || !out->dL_drotations ||
               (f->M > 0 && !out->dL_dsh) ||
               (!raw && (!out->dL_dmeans2D || !out->dL_dcolors || !out->dL_dcov3D)) ||
               (raw && f->M > 1 && !out->dL_dsh_rest)) {
        return fail(RR_ERR_ARG, "null gradient output");
    }
    if (!raw && !out->dL_dopacity) return fail(RR_ERR_ARG, "null gradient output");
    if (out->grad_accum && (!raw || !out->denom || !out->max_radii2D))
        return fail(RR_ERR_ARG, "densification statistics need raw mode and grad_accum, denom, max_radii2D");
    if (workspace_bytes < rr_backward_workspace_bytes(P)) return fail(RR_ERR_CAPACITY, "workspace too small");
    const rr_next_frame* nx = out->next;
    if (nx) {  // cross-step fusion: the next frame's preprocess on the stepped parameters
        if (!ad) return fail(RR_ERR_ARG, "rr_grads.next needs the fused optimizer step (rr_grads.adam)");
        if (!nx->frame || !nx->cam || !nx->radii || !nx->geom_buffer)
            return fail(RR_ERR_ARG, "rr_next_frame: null frame / camera / radii / geometry buffer");
        const rr_frame* nf = nx->frame;
        if (nf->P != P || nf->M != f->M || nf->D != f->D || !(nf->flags & RR_FLAG_RAW_PARAMS) ||
            (nf->flags & RR_FLAG_AUX_NORMAL) || nf->prefiltered)
            return fail(RR_ERR_ARG, "rr_next_frame: the next frame must have the same P, M and SH degree, raw "
                                    "parameters, no aux normals, no prefiltering");
        if (nf->width <= 0 || nf->height <= 0) return fail(RR_ERR_ARG, "rr_next_frame: bad width / height");
        if (!nx->cam->viewmatrix || !nx->cam->projmatrix || !nx->cam->campos)
            return fail(RR_ERR_ARG, "rr_next_frame: camera arrays are required");
        if (nx->geom_bytes < carve_geom(nullptr, P).total) return fail(RR_ERR_CAPACITY, "next geometry buffer too small");
        if (nx->geom_buffer == geom_buffer) return fail(RR_ERR_ARG, "rr_next_frame: the next frame needs its own geometry buffer");
        const rr_adam_group* gs[6] = {&ad->xyz, &ad->f_dc, &ad->f_rest, &ad->opacity, &ad->scaling, &ad->rotation};
        for (int i = 0; i < 6; i++)
            if (!gs[i]->param && !(i == 2 && f->M <= 1))
                return fail(RR_ERR_ARG, "rr_next_frame: every Adam group must be stepped");
    }
    hipStream_t st = (hipStream_t)stream;
    float* gacc = static_cast<float*>(workspace);
    if (int rc2 = blend_backward(f, cam, geom_buffer, image_buffer, binning_buffer, L, dL_dpix, gacc, st)) return rc2;
    {
        StageTimer tm(RR_STAGE_GAUSS_BWD, st);
        GaussBwdArgs a{};
        a.P = P; a.D = f->D; a.M = f->M;
        a.tanfovx = f->tan_fovx; a.tanfovy = f->tan_fovy;
        a.focal_y = H / (2.0f * f->tan_fovy);
        a.focal_x = W / (2.0f * f->tan_fovx);
        a.scale_modifier = f->scale_modifier; a.low_pass = f->low_pass;
        a.means3D = g->means3D; a.shs = g->shs; a.scales = g->scales; a.rotations = g->rotations;
        a.cov3D_precomp = g->cov3D_precomp; a.view = cam->viewmatrix; a.proj = cam->projmatrix;
        a.campos = cam->campos; a.radii = radii; a.gacc = gacc;
        a.dL_dmeans2D = out->dL_dmeans2D; a.dL_dcolors = out->dL_dcolors; a.dL_dopacity = out->dL_dopacity;
        a.dL_dmeans3D = out->dL_dmeans3D; a.dL_dcov3D = out->dL_dcov3D; a.dL_dsh = f->M > 0 ? out->dL_dsh : nullptr;
        a.dL_dscales = out->dL_dscales; a.dL_drot = out->dL_drotations;
        a.raw = raw ? 1 : 0; a.opacities = g->opacities; a.shs_rest = g->shs_rest;
        a.dL_dsh_rest = out->dL_dsh_rest;
        a.grad_accum = out->grad_accum; a.denom = out->denom; a.max_radii2D = out->max_radii2D;
        a.use_adam = ad ? 1 : 0;
        if (ad) a.adam = *ad;  // by value: the kernel must not dereference host memory
        if (nx) {
            const Geom ng = carve_geom(nx->geom_buffer, P);
            PreArgs n = pre_args(nx->frame, nx->cam, g);
            n.radii = nx->radii; n.splats = ng.splats; n.tiles = ng.tiles; n.depth_keys = ng.depth_keys;
            n.block_sums = ng.block_sums; n.block_wide = ng.block_wide; n.n_out = P;
            a.next = n;
            a.has_next = 1;
        }
        launch_gauss_bwd(a, st);
    }
    RR_STAGE_CHECK("gaussian backward");
    return RR_OK;
}

// ---- Gaussian-sharded multi-GPU step (include/rain_raster.h, "row blocks") ----

int rr_geometry_layout(int P, size_t* offsets) {
    if (P < 0 || !offsets) return fail(RR_ERR_ARG, "bad P / null offsets");
    // carve over a stand-in base address (a null base carves null pointers) and subtract it
    constexpr uintptr_t kBase = 1u << 20;
    const Geom gm = carve_geom(reinterpret_cast<void*>(kBase), P);
    auto off = [](const void* p) { return (size_t)(reinterpret_cast<uintptr_t>(p) - kBase); };
    offsets[0] = off(gm.splats);
    offsets[1] = off(gm.tiles);
    offsets[2] = off(gm.depth_keys);
    offsets[3] = off(gm.block_sums);
    offsets[4] = off(gm.block_wide);
    return RR_OK;
}

int rr_preprocess_rows(const rr_frame* f, const rr_camera* cam, const rr_gaussians* g, int n_rows, int* radii,
                       void* splats, void* tiles, void* depth_keys, void* block_sums, void* block_wide, void* stream) {
    int rc = validate(f, cam, g, true);
    if (rc) return rc;
    if (n_rows < f->P || (n_rows % 256) != 0) return fail(RR_ERR_ARG, "n_rows must be >= P and a multiple of 256");
    if (n_rows == 0) return RR_OK;
    if (!radii || !splats || !tiles || !depth_keys || !block_sums || !block_wide)
        return fail(RR_ERR_ARG, "null output array");
    if (f->flags & RR_FLAG_AUX_NORMAL) return fail(RR_ERR_ARG, "row blocks carry no aux normals");
    hipStream_t st = (hipStream_t)stream;
    PreArgs a = pre_args(f, cam, g);
    a.radii = radii;
    a.splats = static_cast<Splat*>(splats);
    a.tiles = static_cast<uint2*>(tiles);
    a.depth_keys = static_cast<uint32_t*>(depth_keys);
    a.block_sums = static_cast<uint2*>(block_sums);
    a.block_wide = static_cast<uint32_t*>(block_wide);
    a.n_out = n_rows;
    {
        StageTimer tm(RR_STAGE_PREPROCESS, st);
        launch_preprocess(a, st);
    }
    RR_STAGE_CHECK("preprocess (rows)");
    return RR_OK;
}

int rr_preprocess_rows_views(const rr_frame* f, const rr_view* views, int num_views, const rr_gaussians* g,
                             int n_rows, void* out, size_t view_stride, const size_t field_offsets[6], int wire,
                             void* stream) {
    if (!f || !views || !g || !field_offsets) return fail(RR_ERR_ARG, "null argument");
    if (num_views < 1 || num_views > RR_MAX_VIEWS) return fail(RR_ERR_ARG, "1 <= num_views <= RR_MAX_VIEWS");
    if (n_rows < f->P || (n_rows % 256) != 0) return fail(RR_ERR_ARG, "n_rows must be >= P and a multiple of 256");
    if (f->flags & RR_FLAG_AUX_NORMAL) return fail(RR_ERR_ARG, "row blocks carry no aux normals");
    for (int v = 0; v < num_views; v++) {
        const rr_view& w = views[v];
        if (!w.viewmatrix || !w.projmatrix || !w.campos || w.width <= 0 || w.height <= 0)
            return fail(RR_ERR_ARG, "bad view");
    }
    // the frame's own validation, with view 0 standing in for the camera (the preprocess reads no
    // background)
    const rr_camera cam0{views[0].viewmatrix, views[0].viewmatrix, views[0].projmatrix, views[0].campos};
    int rc = validate(f, &cam0, g, true);
    if (rc) return rc;
    if (n_rows == 0) return RR_OK;
    if (!out) return fail(RR_ERR_ARG, "null output buffer");
    PreArgs a = pre_args(f, &cam0, g);
    char* base = static_cast<char*>(out);
    a.radii = reinterpret_cast<int*>(base + field_offsets[0]);
    if (wire) {  // 10-float wire records, no depth keys (rr_unpack_rows rebuilds both)
        if ((field_offsets[1] | view_stride) & 7u) return fail(RR_ERR_ARG, "wire records need 8-B alignment");
        a.wire = reinterpret_cast<float*>(base + field_offsets[1]);
    } else {
        a.splats = reinterpret_cast<Splat*>(base + field_offsets[1]);
        a.depth_keys = reinterpret_cast<uint32_t*>(base + field_offsets[3]);
    }
    a.tiles = reinterpret_cast<uint2*>(base + field_offsets[2]);
    a.block_sums = reinterpret_cast<uint2*>(base + field_offsets[4]);
    a.block_wide = reinterpret_cast<uint32_t*>(base + field_offsets[5]);
    a.n_out = n_rows;
    PreViews vs{};
    vs.V = num_views;
    vs.stride = view_stride;
    for (int v = 0; v < num_views; v++) {
        const rr_view& w = views[v];
        PreView& c = vs.v[v];
        c.view = w.viewmatrix;
        c.proj = w.projmatrix;
        c.campos = w.campos;
        c.tanfovx = w.tan_fovx;
        c.tanfovy = w.tan_fovy;
        c.focal_x = w.width / (2.0f * w.tan_fovx);
        c.focal_y = w.height / (2.0f * w.tan_fovy);
        c.low_pass = w.low_pass;
        c.W = w.width;
        c.H = w.height;
        c.gx = grid_x(w.width);
        c.gy = grid_y(w.height);
    }
    hipStream_t st = (hipStream_t)stream;
    {
        StageTimer tm(RR_STAGE_PREPROCESS, st);
        launch_preprocess_views(a, vs, st);
    }
    RR_STAGE_CHECK("preprocess (rows, views)");
    return RR_OK;
}

int rr_unpack_rows(int world, int rows_per_rank, const void* recv, size_t chunk_bytes, const size_t field_offsets[5],
                   void* geom_buffer, size_t geom_bytes, int* radii, void* stream) {
    if (world < 1 || rows_per_rank < 0 || (rows_per_rank % 256) != 0)
        return fail(RR_ERR_ARG, "world >= 1 and rows_per_rank a multiple of 256");
    if (!field_offsets) return fail(RR_ERR_ARG, "null field offsets");
    const int P = world * rows_per_rank;
    if (P == 0) return RR_OK;
    if (!recv || !geom_buffer || !radii) return fail(RR_ERR_ARG, "null buffer");
    if ((chunk_bytes | field_offsets[0] | field_offsets[1]) & 7u)
        return fail(RR_ERR_ARG, "chunks and wire / tile fields need 8-B alignment");
    const Geom gm = carve_geom(geom_buffer, P);
    if (geom_bytes < gm.total) return fail(RR_ERR_CAPACITY, "geometry buffer too small");
    hipStream_t st = (hipStream_t)stream;
    launch_unpack_rows(world, rows_per_rank, static_cast<const char*>(recv), chunk_bytes, field_offsets, gm.splats,
                       gm.tiles, gm.depth_keys, radii, gm.block_sums, gm.block_wide, st);
    return check(nullptr, st, "unpack rows");
}

int rr_forward_from_geometry(const rr_frame* f, const rr_camera* cam, const int* radii, void* geom_buffer,
                             size_t geom_bytes, void* image_buffer, size_t image_bytes, void* binning_buffer,
                             size_t binning_bytes, int* num_rendered, int* num_pairs, size_t* binning_needed,
                             float* out_color, float* out_depth, void* stream) {
    if (!f || !cam || !num_rendered || !num_pairs || !binning_needed) return fail(RR_ERR_ARG, "null argument");
    *num_rendered = 0;
    *num_pairs = 0;
    *binning_needed = 0;
    const int P = f->P, W = f->width, H = f->height;
    if (P < 0 || W <= 0 || H <= 0) return fail(RR_ERR_ARG, "bad P / width / height");
    if (f->flags & RR_FLAG_AUX_NORMAL) return fail(RR_ERR_ARG, "row blocks carry no aux normals");
    if (P == 0) return RR_OK;
    if (!radii || !geom_buffer || !image_buffer || !out_color || !out_depth || !cam->background)
        return fail(RR_ERR_ARG, "null buffer");
    const Geom gm = carve_geom(geom_buffer, P);
    const Img im = carve_img(image_buffer, W, H);
    if (geom_bytes < gm.total || image_bytes < im.total) return fail(RR_ERR_CAPACITY, "scratch buffer too small");
    hipStream_t st = (hipStream_t)stream;
    if (int rc = count_pairs(f, gm, im, P, st, num_rendered, num_pairs)) return rc;
    const size_t need = *num_pairs > 0 ? carve_bin(nullptr, *num_pairs, W, H).total : 0;
    *binning_needed = need;
    if (binning_bytes < need) return RR_INCOMPLETE;
    return render_frame(f, cam, radii, geom_buffer, image_buffer, binning_buffer, binning_bytes, *num_pairs, out_color,
                        out_depth, nullptr, stream);
}

int rr_forward_render_geometry(const rr_frame* f, const rr_camera* cam, const int* radii, void* geom_buffer,
                               void* image_buffer, void* binning_buffer, size_t binning_bytes, int num_pairs,
                               float* out_color, float* out_depth, void* stream) {
    if (!f || !cam || (f->flags & RR_FLAG_AUX_NORMAL)) return fail(RR_ERR_ARG, "bad frame / camera");
    if (f->P == 0) return RR_OK;
    if (!radii || !cam->background) return fail(RR_ERR_ARG, "null buffer");
    return render_frame(f, cam, radii, geom_buffer, image_buffer, binning_buffer, binning_bytes, num_pairs, out_color,
                        out_depth, nullptr, stream);
}

int rr_backward_records(const rr_frame* f, const rr_camera* cam, const int* radii, const void* geom_buffer,
                        const void* image_buffer, const void* binning_buffer, int num_rendered, const float* dL_dpix,
                        void* workspace, size_t workspace_bytes, int rows_per_rank, int chunk_rows, float* records,
                        void* stream) {
    if (!f || !cam) return fail(RR_ERR_ARG, "null frame / camera");
    const int P = f->P;
    if (P < 0) return fail(RR_ERR_ARG, "bad P");
    if (rows_per_rank < 0 || (rows_per_rank > 0 && (P % rows_per_rank != 0 || chunk_rows < 1)))
        return fail(RR_ERR_ARG, "rows_per_rank must divide P (and chunk_rows >= 1), or be 0");
    if (P == 0) return RR_OK;
    if (!radii || !geom_buffer || !image_buffer || !dL_dpix || !workspace || !records || !cam->background)
        return fail(RR_ERR_ARG, "null buffer");
    if (workspace_bytes < rr_backward_workspace_bytes(P)) return fail(RR_ERR_CAPACITY, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    float* gacc = static_cast<float*>(workspace);
    if (int rc = blend_backward(f, cam, geom_buffer, image_buffer, binning_buffer, num_rendered, dL_dpix, gacc, st))
        return rc;
    launch_pack_records(gacc, radii, P, rows_per_rank, rows_per_rank > 0 ? std::min(chunk_rows, rows_per_rank) : 1,
                        records, st);
    return check(f, st, "pack records");
}

int rr_gauss_backward_views(const rr_frame* f, const rr_view* views, int num_views, const rr_gaussians* g,
                            const float* records, int record_rows, float grad_scale, const rr_grads* out,
                            void* stream) {
    if (!f || !views || !g || !out) return fail(RR_ERR_ARG, "null argument");
    if (num_views < 1 || num_views > RR_MAX_VIEWS) return fail(RR_ERR_ARG, "1 <= num_views <= RR_MAX_VIEWS");
    const int P = f->P;
    if (P < 0 || record_rows < P) return fail(RR_ERR_ARG, "bad P / record_rows");
    if (!(f->flags & RR_FLAG_RAW_PARAMS)) return fail(RR_ERR_ARG, "the sharded backward runs in raw-parameter mode");
    if (f->M < 1 || f->M > 16 || f->D < 0 || f->D > 3 || f->M < (f->D + 1) * (f->D + 1))
        return fail(RR_ERR_ARG, "sh_degree must be 0..3 and M >= (degree+1)^2, M <= 16");
    if (P == 0) return RR_OK;
    if (!records || !g->means3D || !g->shs || !g->opacities || !g->scales || !g->rotations || (f->M > 1 && !g->shs_rest))
        return fail(RR_ERR_ARG, "raw parameters and records are required");
    if (out->dL_dmeans2D || out->dL_dcolors || out->dL_dopacity || out->dL_dmeans3D || out->dL_dcov3D || out->dL_dsh ||
        out->dL_dscales || out->dL_drotations || out->dL_dsh_rest)
        return fail(RR_ERR_ARG, "the sharded backward writes no gradient arrays (Adam and statistics only)");
    if (out->grad_accum && (!out->denom || !out->max_radii2D))
        return fail(RR_ERR_ARG, "densification statistics need grad_accum, denom, max_radii2D");
    const rr_adam* ad = out->adam;
    if (ad) {
        const rr_adam_group* gs[6] = {&ad->xyz, &ad->f_dc, &ad->f_rest, &ad->opacity, &ad->scaling, &ad->rotation};
        const void* in[6] = {g->means3D, g->shs, g->shs_rest, g->opacities, g->scales, g->rotations};
        for (int i = 0; i < 6; i++) {
            if (!gs[i]->param || (i == 2 && f->M <= 1)) continue;  // a group without param is not stepped
            if (!gs[i]->exp_avg || !gs[i]->exp_avg_sq) return fail(RR_ERR_ARG, "null Adam moment array");
            if (gs[i]->param != in[i]) return fail(RR_ERR_ARG, "Adam group param must be the matching input array");
        }
    }
    ViewCam cams[RR_MAX_VIEWS];
    for (int v = 0; v < num_views; v++) {
        const rr_view& w = views[v];
        if (!w.viewmatrix || !w.projmatrix || !w.campos || w.width <= 0 || w.height <= 0)
            return fail(RR_ERR_ARG, "bad view");
        cams[v] = ViewCam{w.viewmatrix, w.projmatrix, w.campos, w.tan_fovx, w.tan_fovy,
                          w.width / (2.0f * w.tan_fovx), w.height / (2.0f * w.tan_fovy), w.low_pass};
    }
    hipStream_t st = (hipStream_t)stream;
    GaussBwdArgs a{};
    a.P = P; a.D = f->D; a.M = f->M;
    a.scale_modifier = f->scale_modifier;
    a.means3D = g->means3D; a.shs = g->shs; a.scales = g->scales; a.rotations = g->rotations;
    a.raw = 1; a.opacities = g->opacities; a.shs_rest = g->shs_rest;
    a.grad_accum = out->grad_accum; a.denom = out->denom; a.max_radii2D = out->max_radii2D;
    a.use_adam = ad ? 1 : 0;
    if (ad) a.adam = *ad;
    {
        StageTimer tm(RR_STAGE_GAUSS_BWD, st);
        if (launch_gauss_bwd_views(a, cams, num_views, records, record_rows, grad_scale, st))
            return fail(RR_ERR_ARG, "bad number of views");
    }
    return check(f, st, "gaussian backward (views)");
}

int rr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix, uint8_t* present,
                    void* stream) {
    (void)projmatrix;
    if (P < 0) return fail(RR_ERR_ARG, "bad P");
    if (P == 0) return RR_OK;
    if (!means3D || !viewmatrix || !present) return fail(RR_ERR_ARG, "null pointer");
    hipStream_t st = (hipStream_t)stream;
    launch_mark_visible(P, means3D, viewmatrix, present, st);
    return check(nullptr, st, "mark_visible");
}

int rr_read_frame_stats(const rr_frame* f, const void* geom_buffer, const void* image_buffer, rr_frame_stats* out,
                        void* stream) {
    if (!f || !out) return fail(RR_ERR_ARG, "null");
    std::memset(out, 0, sizeof(*out));
    const int P = f->P, W = f->width, H = f->height;
    const int T = grid_x(W) * grid_y(H);
    out->tiles = T;
    if (P == 0) return RR_OK;
    const Geom gm = carve_geom(const_cast<void*>(geom_buffer), P);
    const Img im = carve_img(const_cast<void*>(image_buffer), W, H);
    hipStream_t st = (hipStream_t)stream;
    FrameTotals ft{};
    std::vector<uint32_t> tm(T);
    std::vector<uint2> per((size_t)P);
    RR_CHECK(hipMemcpyAsync(&ft, gm.ft, sizeof(ft), hipMemcpyDeviceToHost, st), "stats");
    RR_CHECK(hipMemcpyAsync(per.data(), gm.tiles, (size_t)P * sizeof(uint2), hipMemcpyDeviceToHost, st), "stats");
    RR_CHECK(hipMemcpyAsync(tm.data(), im.tile_max, (size_t)T * 4, hipMemcpyDeviceToHost, st), "stats");
    // [0] phase-B pairs (the gather path: slots reserved), [2] phase B took the gather path,
    // [3] phase-B pairs the gather path's bin runs hold
    uint32_t cnt[4] = {0u, 0u, 0u, 0u};
    RR_CHECK(hipMemcpyAsync(cnt, im.counters, sizeof(cnt), hipMemcpyDeviceToHost, st), "stats");
    RR_CHECK(hipStreamSynchronize(st), "stats");
    int64_t vis = 0;
    for (const uint2& v : per) vis += v.y > 0;  // a Gaussian is visible iff its rect is non-empty (radii > 0)
    out->num_visible = vis;
    out->num_rendered = (int64_t)ft.rect;
    out->num_pairs = (int64_t)ft.L;
    int64_t s = 0;
    for (uint32_t v : tm) s += v;
    out->l_eff = s;
    // phase A's pairs, and the phase-B pairs kept for the tiles phase A left open (by the path the
    // frame took: its phase-B duplicate marks the gather path in counters[2])
    out->num_binned = (int64_t)ft.LA + (cnt[2] ? cnt[3] : cnt[0]);
    out->phase_b_pairs = (int64_t)ft.LB;
    out->phase_b_slots = (int64_t)cnt[0];
    return RR_OK;
}

int rr_debug_get_views(const rr_frame* f, const void* geom_buffer, const void* image_buffer,
                       const void* binning_buffer, int num_rendered, rr_debug_views* out) {
    if (!f || !out) return fail(RR_ERR_ARG, "null");
    const Geom gm = carve_geom(const_cast<void*>(geom_buffer), f->P);
    const Img im = carve_img(const_cast<void*>(image_buffer), f->width, f->height);
    const Bin bn = carve_bin(const_cast<void*>(binning_buffer), num_rendered, f->width, f->height);
    out->point_list = bn.point_list;
    out->ranges = reinterpret_cast<const uint32_t*>(im.ranges);
    out->tile_max = im.tile_max;
    out->final_T = im.final_T;
    out->n_contrib = im.n_contrib;
    out->splats = reinterpret_cast<const float*>(gm.splats);
    return RR_OK;
}

int rr_debug_set_fwd_trace(void* dev_buf) {
    set_fwd_trace(dev_buf);
    return RR_OK;
}

int rr_set_forward_workspace(void* workspace, size_t bytes) {
    if (workspace && (((uintptr_t)workspace & 15u) != 0 || bytes % 16 != 0))
        return fail(RR_ERR_ARG, "workspace must be 16-byte aligned and a multiple of 16 bytes");
    g_fwd_ws = workspace && bytes ? WsRange{workspace, bytes} : WsRange{};
    return RR_OK;
}

int rr_set_tuning(const char* key, int value) {
    if (!key) return fail(RR_ERR_ARG, "unknown tuning key: (null)");
    const std::string k(key);
    Tuning& tu = tuning();
    const Tuning dflt{};
    if (k == "early_den") tu.early_den = value > 0 ? (uint32_t)value : dflt.early_den;
    else if (k == "pair_scan_direct_blocks") tu.pair_scan_direct_blocks = value >= 0 ? value : dflt.pair_scan_direct_blocks;
    else if (k == "wide_bin_keys") tu.wide_bin_keys = value != 0;
    else if (k == "phase_b_gather") tu.b_gather = value != 0;
    else if (k == "dup_b_rows") tu.dup_b_rows = value != 0;
    else if (k == "dup_big_bins") tu.dup_big_bins = value >= 0 ? value : dflt.dup_big_bins;
    else if (k == "sx_bucket") tu.sx_bucket = value != 0;
    else if (k == "sx_lds_cap") tu.sx_lds_cap = value > 0 ? value : 0;
    else if (k == "sort_min_units") tu.sort_min_units = value > 0 ? value : dflt.sort_min_units;
    else if (k == "sort_min_units_tile") tu.sort_min_units_tile = value > 0 ? value : dflt.sort_min_units_tile;
    else if (k == "sort_max_rounds")
        tu.sort_max_rounds = (value == 1 || value == 2 || value == 4 || value == 8) ? value : dflt.sort_max_rounds;
    else return fail(RR_ERR_ARG, "unknown tuning key: " + k);
    return RR_OK;
}

int rr_set_binning_config(int split_denominator, int min_pairs) {
    if (split_denominator < 0 || min_pairs < 0) return fail(RR_ERR_ARG, "negative binning config");
    Tuning& tu = tuning();
    const Tuning dflt{};
    tu.early_den = split_denominator == 0 ? dflt.early_den : (uint32_t)split_denominator;
    tu.early_min = min_pairs == 0 ? dflt.early_min : (uint32_t)min_pairs;
    return RR_OK;
}

int rr_profile_enable(int enable) {
    g_prof = enable != 0;
    return RR_OK;
}

int rr_profile_select(unsigned stage_mask) {
    g_prof_mask = stage_mask;
    return RR_OK;
}

int rr_host_wait_stats(int reset, int64_t* wait_ns, int64_t* waits) {
    if (wait_ns) *wait_ns = g_wait_ns;
    if (waits) *waits = g_waits;
    if (reset) g_wait_ns = g_waits = 0;
    return RR_OK;
}

int rr_profile_collect(double* ms, int64_t* counts) {
    for (auto& r : g_recs) {
        RR_CHECK(hipEventSynchronize(r.b), "profile sync");
        float e = 0.f;
        RR_CHECK(hipEventElapsedTime(&e, r.a, r.b), "profile elapsed");
        if (ms) ms[r.stage] += e;
        if (counts) counts[r.stage] += 1;
        g_pool.push_back(r.a);
        g_pool.push_back(r.b);
    }
    g_recs.clear();
    return RR_OK;
}

const char* rr_stage_name(int stage) {
    static const char* names[RR_NUM_STAGES] = {"preprocess", "depth_sort", "scan", "duplicate", "tile_sort",
                                               "ranges", "blend_fwd", "blend_bwd", "gauss_bwd", "memset"};
    return (stage >= 0 && stage < RR_NUM_STAGES) ? names[stage] : "?";
}

}  // extern "C"
