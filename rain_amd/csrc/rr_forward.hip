// rr_forward.hip — forward kernels of the MI355X rasterizer.
//
//   k_preprocess<DEG>  one thread per Gaussian (forward.cu:144-246 semantics; rr_preprocess.hpp)
//   k_duplicate<K>     (bin, Gaussian) pairs of one early-stop phase in Gaussian index order, key =
//                      bin id only, value = Gaussian | tile mask << BIN_SHIFT (LDS windows; bins:
//                      rr_common.hpp)
//   k_mark_visible     frustum test (rasterizer_impl.cu:43-55)
//
// Binning order: the reference sorts 64-bit (tile << 32 | depth_bits) keys emitted in Gaussian
// index order with a stable radix sort.  Here the pairs are emitted in index order too, stable-
// sorted by bin id only (rr_sort.hip, <= 16-bit keys), and each bin's run is then stable-sorted by
// depth inside one workgroup (rr_bin.hip k_sortexpand) and split into its four tiles' lists.
// Within a tile this yields the reference's (depth, index) order, without a sort of 64-bit keys
// and without a per-frame depth sort of the Gaussians.
#include "rr_common.hpp"
#include "rr_kernels.hpp"
#include "rr_preprocess.hpp"

namespace rr {

// No global atomics here: per-Gaussian counts go to tiles[idx] = {pairs, rect area} (the rect-area
// sum is the reference's num_rendered).  The arithmetic is rr_preprocess.hpp's preprocess_finish.
template <int DEG>
__device__ __forceinline__ uint2 preprocess_one(const PreArgs& a, int idx, bool& wide) {
    preprocess_clear(a, idx);
    const v3 p = load3(a.means3D + 3 * (size_t)idx);
    // in_frustum (auxiliary.h:128-153)
    const v3 p_view = xform_point_4x3(p, a.view);
    if (p_view.z <= 0.2f) {
        if (a.prefiltered) __builtin_trap();
        return make_uint2(0u, 0u);
    }
    // The row's remaining inputs (but the SH coefficients) in one batch right after the depth
    // test: a wave then waits for one memory round trip where it waited for three (rotation and
    // scale, colour, opacity): preprocess 0.080 -> 0.077 ms/step in an interleaved A/B (the SH rows
    // too: 158 VGPRs, 3 waves/SIMD, 0.086; profiles/r03_preprocess_early_ab.jsonl)
    float4 q = make_float4(1.f, 0.f, 0.f, 0.f);
    v3 sc = mk(0.f, 0.f, 0.f);
    if (!a.cov3D_precomp) {
        q = *reinterpret_cast<const float4*>(a.rotations + 4 * (size_t)idx);
        sc = load3(a.scales + 3 * (size_t)idx);
    }
    const float o_in = a.opacities[idx];
    const float* dc = a.raw ? a.shs + 3 * (size_t)idx : a.shs + (size_t)idx * a.M * 3;
    const v3 c0 = load3(a.colors_precomp ? a.colors_precomp + 3 * (size_t)idx : dc);
    const float* rest = a.raw ? a.shs_rest + (size_t)idx * (a.M - 1) * 3 : dc + 3;
    return preprocess_finish<DEG, true>(a, idx, p, p_view, q, sc, o_in, c0, rest, wide);
}

// The block's sums of {pairs, rect tiles} go to a.block_sums[blockIdx.x] (plain stores; a single
// contended 64-bit atomic per block measured +37 us on 1M Gaussians).
template <int DEG>
__device__ __forceinline__ void preprocess_block(const PreArgs& a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    bool wide = false;
    uint2 c = make_uint2(0u, 0u);
    if (idx < a.P) {
        c = preprocess_one<DEG>(a, idx, wide);
    } else if (idx < a.n_out) {  // padding row of a row block: culled
        preprocess_clear(a, idx);
    }
    if (!a.block_sums) return;
    preprocess_block_sums(a, blockIdx.x, c, wide);
}

// 5 waves per SIMD: the SH-3 instance fits 88 VGPRs without spills (the compiler's own choice,
// 98, gives 4; 6 waves spill 52 B/lane): preprocess 0.094 -> 0.090 ms/step in an interleaved A/B
// (profiles/r03_preprocess_occupancy_ab.txt; 8 waves measured 0.129 vs 0.091 in round 2)
#ifndef RR_PRE_OCC
#define RR_PRE_OCC 5
#endif
template <int DEG>
__global__ __launch_bounds__(256, RR_PRE_OCC) void k_preprocess(PreArgs a) {
    preprocess_block<DEG>(a);
}

template <int DEG>
__global__ __launch_bounds__(256, RR_PRE_OCC) void k_preprocess_views(PreArgs a, PreViews vs) {
    const PreView& c = vs.v[blockIdx.y];
    PreArgs b = a;
    b.view = c.view;
    b.proj = c.proj;
    b.campos = c.campos;
    b.tanfovx = c.tanfovx;
    b.tanfovy = c.tanfovy;
    b.focal_x = c.focal_x;
    b.focal_y = c.focal_y;
    b.low_pass = c.low_pass;
    b.W = c.W;
    b.H = c.H;
    b.gx = c.gx;
    b.gy = c.gy;
    const size_t off = (size_t)blockIdx.y * vs.stride;
    auto at = [&](auto* p) { return reinterpret_cast<decltype(p)>(reinterpret_cast<char*>(p) + off); };
    b.radii = at(a.radii);
    b.splats = at(a.splats);
    b.tiles = at(a.tiles);
    b.depth_keys = a.depth_keys ? at(a.depth_keys) : nullptr;
    b.block_sums = at(a.block_sums);
    b.block_wide = at(a.block_wide);
    b.wire = a.wire ? at(a.wire) : nullptr;
    preprocess_block<DEG>(b);
}

// The receiving side of the sharded step's geometry exchange: rows of `world` chunks (chunk j =
// rank j's rows, wire format) into the geometry arrays in global row order, splats rebuilt with
// splat_derived, depth keys from the depth (0xffffffff for a culled row, radius 0).
__global__ __launch_bounds__(256) void k_unpack_rows(int world, int Q, const char* __restrict__ recv, size_t chunk,
                                                     size_t o_wire, size_t o_tiles, size_t o_radii, size_t o_bsum,
                                                     size_t o_bwide, Splat* __restrict__ splats,
                                                     uint2* __restrict__ tiles, uint32_t* __restrict__ keys,
                                                     int* __restrict__ radii, uint2* __restrict__ bsum,
                                                     uint32_t* __restrict__ bwide) {
    const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= (size_t)world * Q) return;
    const int j = (int)(g / (size_t)Q), r = (int)(g - (size_t)j * Q);
    const char* c = recv + (size_t)j * chunk;
    const float2* w = reinterpret_cast<const float2*>(c + o_wire) + (size_t)(kWireFloats / 2) * r;
    const int radius = reinterpret_cast<const int*>(c + o_radii)[r];
    tiles[g] = reinterpret_cast<const uint2*>(c + o_tiles)[r];
    radii[g] = radius;
    Splat s;
    if (radius > 0) {
        const float2 w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
        float log2o, inv_o;
        splat_derived(w3.x, log2o, inv_o);
        s.a = make_float4(w0.x, w0.y, w1.x, w1.y);
        s.b = make_float4(w2.x, log2o, w2.y, w3.x);
        s.c = make_float4(w3.y, w4.x, w4.y, inv_o);
    } else {
        // a culled row's wire record was never written by its owner (the preprocess returns before
        // the record): a zero record keeps the geometry buffer deterministic
        s.a = s.b = s.c = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    splats[g] = s;
    keys[g] = radius > 0 ? __float_as_uint(s.b.z) - kDepthKeyBase : 0xffffffffu;
    if ((r & 255) == 0) {  // Q is a multiple of 256: rank j's block b is global block g / 256
        bsum[g / 256] = reinterpret_cast<const uint2*>(c + o_bsum)[r / 256];
        bwide[g / 256] = reinterpret_cast<const uint32_t*>(c + o_bwide)[r / 256];
    }
}

void launch_unpack_rows(int world, int rows_per_rank, const char* recv, size_t chunk_bytes,
                        const size_t field_offsets[5], Splat* splats, uint2* tiles, uint32_t* depth_keys, int* radii,
                        uint2* block_sums, uint32_t* block_wide, hipStream_t st) {
    const size_t n = (size_t)world * rows_per_rank;
    if (n == 0) return;
    k_unpack_rows<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
        world, rows_per_rank, recv, chunk_bytes, field_offsets[0], field_offsets[1], field_offsets[2],
        field_offsets[3], field_offsets[4], splats, tiles, depth_keys, radii, block_sums, block_wide);
}


// First list entry of every window of `win` consecutive pairs starting at pair0: window k =
// [pair0 + k*win, pair0 + (k+1)*win) starts inside the pair range [a, b) of exactly one entry.
// A second window set (over a second list: the phase-B windows; nwin_b = 0: none) is marked in the
// same pass.  List lengths come from the device (n / n_b); the grid covers the capacity.
__global__ __launch_bounds__(256) void k_window_starts(const uint32_t* __restrict__ n_dev, const uint32_t* __restrict__ off,
                                                       uint32_t pair0, uint32_t win, int nwin,
                                                       uint32_t* __restrict__ first, const uint32_t* __restrict__ n_dev_b,
                                                       const uint32_t* __restrict__ off_b, uint32_t pair0_b,
                                                       uint32_t win_b, int nwin_b, uint32_t* __restrict__ first_b,
                                                       uint32_t* __restrict__ zero, int nzero) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = s; i < nzero; i += gridDim.x * blockDim.x) zero[i] = 0u;
    auto mark = [&](const uint32_t* o, uint32_t p0, uint32_t w, int nw, uint32_t* f) {
        const uint32_t a = s == 0 ? 0u : o[s - 1], b = o[s];
        if (nw <= 0 || a == b || b <= p0) return;
        const uint32_t k0 = a <= p0 ? 0u : (a - p0 + w - 1) / w;
        for (uint32_t k = k0; k <= (b - 1 - p0) / w && k < (uint32_t)nw; k++) f[k] = (uint32_t)s;
    };
    if (nwin > 0 && (uint32_t)s < *n_dev) mark(off, pair0, win, nwin, first);
    if (nwin_b > 0 && (uint32_t)s < *n_dev_b) mark(off_b, pair0_b, win_b, nwin_b, first_b);
}

// duplicateWithKeys (rasterizer_impl.cu:59-100), output-driven: workgroup k produces exactly the
// pairs [pair0 + k*win, pair0 + (k+1)*win) of the phase's index-ordered pair list (offsets .x for
// phase A, .y for phase B: rr_bin.hip's split scan).  Its Gaussians (from first[k] on) emit into an
// LDS window, which then leaves with coalesced stores — the
// per-Gaussian form scatters every pair to its own cache line — and the window's histogram of
// the lowest `dbits` key bits is written as the tile sort's first-pass digit counts (rr_sort.hip
// units == windows).  Output of window k goes to [k*win, ...) of keys / vals.
//
// Phase B of early-stop binning (open_bits != nullptr): only pairs whose tile is still open are
// kept.  A Gaussian whose tile rectangle holds no open tile (its rows' words of the open-tile
// bitmask, from LDS) is skipped without enumerating its bins; the kept pairs of the window are
// compacted (order preserved) and the window's length goes to unit_len[k] (a sparse sort unit) and
// into *n_total.  (A two-pass variant — count the kept pairs, one block scan per round, then write
// them compacted — measured slower: 0.104 vs 0.083 ms/step for both duplicate launches.)
template <typename K, bool FILTER>
__global__ __launch_bounds__(256) void k_duplicate(const uint32_t* __restrict__ n_dev, const uint32_t* __restrict__ idx,
                                                   const uint32_t* __restrict__ offsets,
                                                   const Splat* __restrict__ splats, const int* __restrict__ radii,
                                                   int gx, int gy, int cull, const uint32_t* __restrict__ first,
                                                   uint32_t pair0, uint32_t win, const uint32_t* __restrict__ L_dev,
                                                   K* __restrict__ keys,
                                                   uint32_t* __restrict__ vals, int dbits,
                                                   uint32_t* __restrict__ counts, int units,
                                                   const uint32_t* __restrict__ open_bits,
                                                   uint32_t* __restrict__ unit_len, uint32_t* __restrict__ n_total,
                                                   const uint32_t* __restrict__ order_cost, uint32_t* __restrict__ order_out,
                                                   uint32_t* __restrict__ order_flag, int order_T) {
    // the extra workgroup (block-uniform) is block 0, so that it is dispatched first and runs
    // under the duplicate instead of after it; the windows are blocks 1..units
    if (FILTER && order_out && blockIdx.x == 0) {
        tile_order_body256(order_T, order_cost, open_bits, order_out);
        if (threadIdx.x == 0) *order_flag = (uint32_t)order_T;
        return;
    }
    const int wb = (FILTER && order_out) ? (int)blockIdx.x - 1 : (int)blockIdx.x;  // window
    // open-tile bitmask in LDS for grids of <= 65536 tiles; larger grids read open_bits directly
    // (FILTER: phase B; the unfiltered kernel does without the mask's 8 KiB of LDS)
    const bool kMaskLds = FILTER && gx * gy <= 65536;
    __shared__ K s_key[kSortMaxUnit];
    __shared__ uint32_t s_val[kSortMaxUnit];
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_open[FILTER ? 2048 : 1];
    __shared__ uint32_t wsum[4];
    const int t = threadIdx.x;
    const int ndig = 1 << dbits;
    constexpr bool filter = FILTER;
    for (int d = t; d < ndig; d += 256) hist[d] = 0;
    // the phase's pair count is device-side: the grid covers the frame's total, and a window past
    // the phase's end is empty (zero counts, zero length)
    const uint32_t L = *L_dev;
    const uint32_t w0 = pair0 + wb * win, w1 = max(w0, min(w0 + win, L));
    const uint32_t wn = w1 - w0;
    if (filter) {
        for (uint32_t j = t; j < wn; j += 256) s_val[j] = 0xffffffffu;  // not emitted
        if (kMaskLds)
            for (int i = t; i < (gx * gy + 31) / 32; i += 256) s_open[i] = open_bits[i];
        __syncthreads();
    }
    auto is_open = [&](uint32_t tile) -> bool {
        const uint32_t word = kMaskLds ? s_open[tile >> 5] : open_bits[tile >> 5];
        return ((word >> (tile & 31)) & 1u) != 0;
    };
    // the bin's tiles still open (phase B), as a bin mask
    auto open4 = [&](int X, int Y) -> uint32_t {
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int tx = 2 * X + (b & 1), ty = 2 * Y + (b >> 1);
            if (tx < gx && ty < gy && is_open((uint32_t)(ty * gx + tx))) m |= 1u << b;
        }
        return m;
    };
    // any open tile in the rectangle [x0, x1) x [y0, y1): the bitmask words of each row, first hit
    // ends the walk (rows are contiguous bit runs: usually one or two words per row)
    auto rect_open = [&](int x0, int y0, int x1, int y1) -> bool {
        for (int y = y0; y < y1; y++) {
            const uint32_t lo = (uint32_t)(y * gx + x0), hi = (uint32_t)(y * gx + x1);  // bits [lo, hi)
            for (uint32_t wd = lo >> 5; wd <= (hi - 1) >> 5; wd++) {
                uint32_t m = kMaskLds ? s_open[wd] : open_bits[wd];
                if (wd == lo >> 5) m &= ~0u << (lo & 31);
                if (wd == (hi - 1) >> 5) m &= ~0u >> (31 - ((hi - 1) & 31));
                if (m) return true;
            }
        }
        return false;
    };
    const int bgx = bins_x(gx);
    const int s0 = (int)first[wb];
    const int P = (int)*n_dev;  // entries of the phase's list
    for (int base = s0; wn > 0; base += 256) {
        const int s = base + t;
        if (s < P) {
            // two dependent load steps per Gaussian: {offsets, index} then {radius, record} (the
            // index is part of the branch condition and the culling setup precedes the open-tile
            // test, so the compiler cannot sink these loads behind a wait into the branches)
            const uint32_t a = s == 0 ? 0u : offsets[s - 1], b = offsets[s];
            const uint32_t g = idx[s];
            const uint32_t lo = max(a, w0), hi = min(b, w1);
            if (lo < hi) {
                const int r = radii[g];
                const float4 A = splats[g].a;
                const float4 Bv = splats[g].b;
                // all of the record in one round trip (the compiler otherwise fetches part of it
                // only after waiting for the rest)
                asm volatile("" ::"v"(r), "v"(A.x), "v"(A.y), "v"(A.z), "v"(A.w), "v"(Bv.x), "v"(Bv.w));
                float ccx, ccy, ccz;
                splat_conic(A, Bv, ccx, ccy, ccz);
                const CullEll ell = cull_setup(A.x, A.y, ccx, ccy, ccz, cull ? cull_qmax(Bv.w) : 0.f);
                int x0, y0, x1, y1;
                tile_rect(A.x, A.y, r, gx, gy, x0, y0, x1, y1);
                const bool any_open = !filter || (x0 < x1 && y0 < y1 && rect_open(x0, y0, x1, y1));
                if (any_open) {
                    uint32_t pos = a;
                    for (int Y = y0 >> 1; Y < (y1 + 1) >> 1 && pos < hi; Y++) {
                        int l0, h0, l1, h1, Xa, Xb;
                        bin_row_spans(ell, cull, Y, x0, x1, y0, y1, l0, h0, l1, h1);
                        bin_cols(l0, h0, l1, h1, Xa, Xb);
                        const uint32_t c = bin_count(l0, h0, l1, h1);
                        if (pos + c <= lo) {  // bin row entirely before the window
                            pos += c;
                            continue;
                        }
                        for (int X = Xa; X < Xb && pos < hi; X++) {
                            uint32_t m = bin_mask(X, l0, h0, l1, h1);
                            if (!m) continue;
                            if (pos >= lo) {
                                if (filter) m &= open4(X, Y);
                                if (m) {
                                    s_key[pos - w0] = (K)(Y * bgx + X);
                                    s_val[pos - w0] = g | (m << BIN_SHIFT);
                                }
                            }
                            pos++;
                        }
                    }
                }
            }
        }
        // another round only if this round's last Gaussian ends before the window does
        const int last = min(base + 255, P - 1);
        if (last >= P - 1 || offsets[last] >= w1) break;
    }
    __syncthreads();
    const uint32_t mask = (uint32_t)ndig - 1u;
    K* const kout = keys + (size_t)wb * win;
    uint32_t* const vout = vals + (size_t)wb * win;
    if (!filter) {
        for (uint32_t j = t; j < wn; j += 256) {
            const K k = s_key[j];
            kout[j] = k;
            vout[j] = s_val[j];
            atomicAdd(&hist[(uint32_t)k & mask], 1u);
        }
    } else {
        // order-preserving compaction in rounds of 256 slots: wave ballots give each kept pair its
        // rank inside the round, the four wave totals the round's block offsets
        const int lane = t & 63, wv = t >> 6;
        const uint64_t lt = (1ull << lane) - 1ull;
        uint32_t carry = 0;
        for (uint32_t r0 = 0; r0 < wn; r0 += 256) {
            const uint32_t j = r0 + t;
            const uint32_t v = j < wn ? s_val[j] : 0xffffffffu;
            const bool kept = v != 0xffffffffu;
            const uint64_t m = __ballot(kept);
            if (lane == 0) wsum[wv] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t pre = carry, tot = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                pre += i < wv ? wsum[i] : 0u;
                tot += wsum[i];
            }
            if (kept) {
                const K k = s_key[j];
                const uint32_t pos = pre + (uint32_t)__popcll(m & lt);
                kout[pos] = k;
                vout[pos] = v;
                atomicAdd(&hist[(uint32_t)k & mask], 1u);
            }
            carry += tot;
            __syncthreads();
        }
        if (t == 0) {
            unit_len[wb] = carry;
            if (carry) atomicAdd(n_total, carry);
        }
    }
    __syncthreads();
    for (int d = t; d < ndig; d += 256) counts[(size_t)d * units + wb] = hist[d];
}

// Phase B of early-stop binning by the gather path (the duplicate, rasterizer_impl.cu:59-100): one
// thread per Gaussian of the phase's list (the split scan's, in index order) instead of
// output-driven windows over a pair list, so no window starts and no stable bin sort after it.  It
// keeps only the pairs on tiles phase A left open: a Gaussian whose rectangle holds no open tile is
// done after one record load; the others reserve min(their pair count, their clipped rectangle's
// open bins) slots and fill them with one walk (slots the walk leaves get a key past the last bin,
// which the bin count and scatter skip).  Each workgroup reserves its slots with one atomic on
// *n_total and writes them densely, in no particular order: the per-bin sort (rr_bin.hip
// k_sortexpand) restores the reference's (depth, index) order.  The extra workgroup 0 computes the
// backward's tile order as k_duplicate's does.  Gaussians whose rectangle spans more than big_bins
// bins (default 32) are emitted by their whole workgroup, 256 bins at a time.
namespace {
// bit i of the result: bit 2i or 2i+1 of x (tile columns -> bin columns)
__device__ __forceinline__ uint32_t pair_bits(uint64_t x) {
    x = (x | (x >> 1)) & 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
    return (uint32_t)x;
}
// bits [a - base, b - base) clipped to [0, 64)
__device__ __forceinline__ uint64_t span_bits(int a, int b, int base) {
    a = max(a - base, 0);
    b = min(b - base, 64);
    if (a >= b) return 0ull;
    return (b == 64 ? ~0ull : (1ull << b) - 1ull) & ~((1ull << a) - 1ull);
}
}  // namespace
// rows: phase B's open tiles as row masks (frames up to 128 tiles wide and 256 tall; Tuning::dup_b_rows
// off forces the flat mask of wider frames onto small ones)
template <typename K>
__global__ __launch_bounds__(256) void k_dup_gather(const uint2* __restrict__ tiles, const Splat* __restrict__ splats,
                                                    const int* __restrict__ radii, int gx, int gy, int cull,
                                                    K* __restrict__ keys, uint32_t* __restrict__ vals,
                                                    const uint32_t* __restrict__ open_bits,
                                                    uint32_t* __restrict__ n_total,
                                                    const uint32_t* __restrict__ order_cost,
                                                    uint32_t* __restrict__ order_out,
                                                    uint32_t* __restrict__ order_flag, int order_T,
                                                    const uint32_t* __restrict__ list_n,
                                                    const uint32_t* __restrict__ list_idx, int big_bins, int rows,
                                                    uint32_t* __restrict__ gather_mark) {
    if (gather_mark && blockIdx.x == 0 && threadIdx.x == 0) *gather_mark = 1u;
    if (order_out && blockIdx.x == 0) {
        tile_order_body256(order_T, order_cost, open_bits, order_out);
        if (threadIdx.x == 0) *order_flag = (uint32_t)order_T;
        return;
    }
    const int wb = order_out ? (int)blockIdx.x - 1 : (int)blockIdx.x;
    // the grid covers every Gaussian, the list only the phase's (block-uniform exit before the
    // open-tile mask is staged)
    if (wb * 256 >= (int)*list_n) return;
    const bool mask_lds = gx * gy <= 65536;
    __shared__ uint32_t s_open[2048];
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t s_base;
    __shared__ uint32_t s_big[256];  // Gaussians of > big_bins bins, done by the whole workgroup
    __shared__ uint32_t s_nbig;      // after the per-thread walks
    if (threadIdx.x == 0) s_nbig = 0u;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int s = wb * 256 + t;
    // this thread's Gaussian (entry s of the list: dense lanes) and its pair count (loads first:
    // they overlap the mask's).  The reservation is bounded by the pair count: the counts of the
    // phase's Gaussians sum to its share of the frame total L, so the reservations never pass the
    // end of the phase's region [L, 2L) (a rectangle's open bins alone can: elongated Gaussians
    // whose culled pairs are few, on a frame where phase A closed few tiles)
    uint32_t n = 0u, g = 0u;
    if (s < (int)*list_n) {
        g = list_idx[s];
        n = tiles[g].x;
    }
    const bool in_phase = n > 0u;
    // phase B: the open tiles' bounding box [ox0, ox1) x [oy0, oy1) (phase A leaves a few tiles open,
    // usually in one corner): every Gaussian's rect is clipped to it first, so most are rejected
    // without a mask walk, and the walks and reservations cover only the clipped rect (the clipped
    // spans are the full ones intersected with the box; the tiles cut off are closed)
    int ox0 = 0, oy0 = 0, ox1 = gx, oy1 = gy;
    {
        __shared__ int s_box[4][4];
        int bx0 = gx, by0 = gy, bx1 = 0, by1 = 0;
        for (int i = t; i < (gx * gy + 31) / 32; i += 256) {
            const uint32_t word = open_bits[i];
            if (mask_lds) s_open[i] = word;
            for (uint32_t m = word; m; m &= m - 1u) {
                const int tile = 32 * i + __builtin_ctz(m), ty = tile / gx, tx = tile - ty * gx;
                bx0 = min(bx0, tx);
                bx1 = max(bx1, tx + 1);
                by0 = min(by0, ty);
                by1 = max(by1, ty + 1);
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            bx0 = min(bx0, __shfl_xor(bx0, o));
            bx1 = max(bx1, __shfl_xor(bx1, o));
            by0 = min(by0, __shfl_xor(by0, o));
            by1 = max(by1, __shfl_xor(by1, o));
        }
        if (lane == 0) {
            s_box[w][0] = bx0;
            s_box[w][1] = by0;
            s_box[w][2] = bx1;
            s_box[w][3] = by1;
        }
        // phase A closed every tile (about half the bench frames): nothing to emit, no record loads
        if (!__syncthreads_or(bx1 > 0)) return;
        ox0 = min(min(s_box[0][0], s_box[1][0]), min(s_box[2][0], s_box[3][0]));
        oy0 = min(min(s_box[0][1], s_box[1][1]), min(s_box[2][1], s_box[3][1]));
        ox1 = max(max(s_box[0][2], s_box[1][2]), max(s_box[2][2], s_box[3][2]));
        oy1 = max(max(s_box[0][3], s_box[1][3]), max(s_box[2][3], s_box[3][3]));
    }
    // frames up to 128 tiles wide and 256 tall (rows): the open tiles also as two
    // 64-bit words per tile row (s_trow) and one per bin row (s_brow, bit X: bin column X holds an
    // open tile), so a rect's open test is one masked word pair per tile row and the walk visits
    // only the bins holding an open tile
    const bool rowm = mask_lds && rows && gx <= 128 && gy <= 256;
    __shared__ uint64_t s_trow[512];
    __shared__ uint64_t s_brow[128];
    if (rowm) {  // block-uniform
        const uint32_t nw = (uint32_t)(gx * gy + 31) / 32;
        for (int r = t; r < 2 * gy; r += 256) {
            const int y = r >> 1, h = r & 1, nbits = min(64, gx - 64 * h);
            uint64_t v = 0ull;
            if (nbits > 0) {
                const uint32_t o = (uint32_t)(y * gx + 64 * h), wi = o >> 5, sh = o & 31;
                const uint64_t w01 = (uint64_t)s_open[wi] | ((wi + 1 < nw ? (uint64_t)s_open[wi + 1] : 0ull) << 32);
                const uint64_t w2 = wi + 2 < nw ? (uint64_t)s_open[wi + 2] : 0ull;
                v = (w01 >> sh) | (sh ? w2 << (64 - sh) : 0ull);
                if (nbits < 64) v &= (1ull << nbits) - 1ull;
            }
            s_trow[r] = v;
        }
        __syncthreads();
        for (int Y = t; Y < bins_y(gy); Y += 256) {
            uint64_t lo = s_trow[4 * Y], hi = s_trow[4 * Y + 1];
            if (2 * Y + 1 < gy) {
                lo |= s_trow[4 * Y + 2];
                hi |= s_trow[4 * Y + 3];
            }
            s_brow[Y] = (uint64_t)pair_bits(lo) | ((uint64_t)pair_bits(hi) << 32);
        }
        __syncthreads();
    }
    auto clip = [&](int& x0, int& y0, int& x1, int& y1) {
        x0 = max(x0, ox0);
        y0 = max(y0, oy0);
        x1 = min(x1, ox1);
        y1 = min(y1, oy1);
    };
    auto is_open = [&](uint32_t tile) -> bool {
        const uint32_t word = mask_lds ? s_open[tile >> 5] : open_bits[tile >> 5];
        return ((word >> (tile & 31)) & 1u) != 0;
    };
    auto open4 = [&](int X, int Y) -> uint32_t {
        if (rowm) {  // tile columns 2X, 2X + 1: two adjacent bits of one word (2X even, < 128)
            const int c = 2 * X, hw = c >> 6, b = c & 63;
            const uint64_t r0 = s_trow[4 * Y + hw], r1 = 2 * Y + 1 < gy ? s_trow[4 * Y + 2 + hw] : 0ull;
            return (uint32_t)((r0 >> b) & 3ull) | ((uint32_t)((r1 >> b) & 3ull) << 2);
        }
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int tx = 2 * X + (b & 1), ty = 2 * Y + (b >> 1);
            if (tx < gx && ty < gy && is_open((uint32_t)(ty * gx + tx))) m |= 1u << b;
        }
        return m;
    };
    auto rect_open = [&](int x0, int y0, int x1, int y1) -> bool {
        if (rowm) {
            const uint64_t mlo = span_bits(x0, x1, 0), mhi = span_bits(x0, x1, 64);
            for (int y = y0; y < y1; y++)
                if ((s_trow[2 * y] & mlo) | (s_trow[2 * y + 1] & mhi)) return true;
            return false;
        }
        for (int y = y0; y < y1; y++) {
            const uint32_t lo = (uint32_t)(y * gx + x0), hi = (uint32_t)(y * gx + x1);  // bits [lo, hi)
            for (uint32_t wd = lo >> 5; wd <= (hi - 1) >> 5; wd++) {
                uint32_t m = mask_lds ? s_open[wd] : open_bits[wd];
                if (wd == lo >> 5) m &= ~0u << (lo & 31);
                if (wd == (hi - 1) >> 5) m &= ~0u >> (31 - ((hi - 1) & 31));
                if (m) return true;
            }
        }
        return false;
    };
    // row masks: the bins of the rect's bin rows and columns holding an open tile — an upper bound
    // on the pairs the walk keeps (0: none)
    auto open_bins = [&](int x0, int y0, int x1, int y1) -> uint32_t {
        const uint64_t bm = span_bits(x0 >> 1, (x1 + 1) >> 1, 0);
        uint32_t c = 0;
        for (int Y = y0 >> 1; Y < (y1 + 1) >> 1; Y++) c += (uint32_t)__popcll(s_brow[Y] & bm);
        return c;
    };
    const int bgx = bins_x(gx);
    uint32_t cnt = 0;
    CullEll ell{};
    int x0 = 0, y0 = 0, x1 = 0, y1 = 0, nbins = 0;
    uint32_t bound = 0;  // the rectangle's open bins (row masks)
    bool live = false;
    if (in_phase) {
        const int r = radii[g];
        const float4 A = splats[g].a;
        const float4 Bv = splats[g].b;
        asm volatile("" ::"v"(r), "v"(A.x), "v"(A.y), "v"(A.z), "v"(A.w), "v"(Bv.x), "v"(Bv.w));
        tile_rect(A.x, A.y, r, gx, gy, x0, y0, x1, y1);
        clip(x0, y0, x1, y1);
        nbins = (((x1 + 1) >> 1) - (x0 >> 1)) * (((y1 + 1) >> 1) - (y0 >> 1));
        if (big_bins > 0 && x0 < x1 && y0 < y1 && nbins > big_bins) {
            s_big[atomicAdd(&s_nbig, 1u)] = g;  // one thread's walk would hold up its workgroup
        } else if (x0 < x1 && y0 < y1 && (rowm ? (bound = open_bins(x0, y0, x1, y1)) > 0u : true) &&
                   rect_open(x0, y0, x1, y1)) {
            float ccx, ccy, ccz;
            splat_conic(A, Bv, ccx, ccy, ccz);
            ell = cull_setup(A.x, A.y, ccx, ccy, ccz, cull ? cull_qmax(Bv.w) : 0.f);
            live = true;
        }
    }
    // Pair i of the workgroup's reservation (at s_base): with the row masks, the first kStage go
    // through LDS (the flat mask's words, no longer read) and out in coalesced rows — each thread's
    // pairs are contiguous, so direct stores scatter 64 runs per instruction — the rest directly
    constexpr uint32_t kStage = 1024u;
    uint32_t* const st_val = s_open;
    uint32_t* const st_key = s_open + kStage;
    auto put = [&](uint32_t i, K key, uint32_t val) {
        if (rowm && i < kStage) {
            st_key[i] = (uint32_t)key;
            st_val[i] = val;
        } else {
            keys[s_base + i] = key;
            vals[s_base + i] = val;
        }
    };
    // the kept pairs, in the duplicate's enumeration (bin rows, then bin columns), at most cap
    auto walk = [&](uint32_t pos, uint32_t cap) {
        uint32_t c = 0;
        if (rowm) {  // block-uniform: only the bin columns of each row that hold an open tile
            const uint64_t bm = span_bits(x0 >> 1, (x1 + 1) >> 1, 0);
            for (int Y = y0 >> 1; Y < (y1 + 1) >> 1 && c < cap; Y++) {
                const uint64_t cand = s_brow[Y] & bm;
                if (!cand) continue;
                int l0, h0, l1, h1, Xa, Xb;
                bin_row_spans(ell, cull, Y, x0, x1, y0, y1, l0, h0, l1, h1);
                bin_cols(l0, h0, l1, h1, Xa, Xb);
                for (uint64_t cm = cand & span_bits(Xa, Xb, 0); cm && c < cap; cm &= cm - 1ull) {
                    const int X = __builtin_ctzll(cm);
                    const uint32_t m = bin_mask(X, l0, h0, l1, h1) & open4(X, Y);
                    if (!m) continue;
                    put(pos + c, (K)(Y * bgx + X), g | (m << BIN_SHIFT));
                    c++;
                }
            }
            return c;
        }
        for (int Y = y0 >> 1; Y < (y1 + 1) >> 1 && c < cap; Y++) {
            // a bin row whose two tile rows hold no open tile in [x0, x1) emits nothing (skipped
            // before its culling spans are evaluated)
            if (!rect_open(x0, max(2 * Y, y0), x1, min(2 * Y + 2, y1))) continue;
            int l0, h0, l1, h1, Xa, Xb;
            bin_row_spans(ell, cull, Y, x0, x1, y0, y1, l0, h0, l1, h1);
            bin_cols(l0, h0, l1, h1, Xa, Xb);
            for (int X = Xa; X < Xb && c < cap; X++) {
                uint32_t m = bin_mask(X, l0, h0, l1, h1);
                m &= open4(X, Y);
                if (!m) continue;
                put(pos + c, (K)(Y * bgx + X), g | (m << BIN_SHIFT));
                c++;
            }
        }
        return c;
    };
    // an upper bound on the kept pairs reserved (the pair count, or the clipped rectangle's open
    // bins or bins if fewer), the slots the one walk leaves filled with a key past the last bin
    if (live) cnt = min(n, rowm ? bound : (uint32_t)nbins);
    // the workgroup's kept pairs: wave prefix sums, one reservation
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        pre += i < w ? wsum[i] : 0u;
        tot += wsum[i];
    }
    if (tot != 0) {  // block-uniform
        if (t == 0) s_base = atomicAdd(n_total, tot);
        __syncthreads();
        if (cnt) {
            const uint32_t pos = pre + incl - cnt;  // in the workgroup's reservation
            const K fill = (K)(bgx * bins_y(gy));
            for (uint32_t c = walk(pos, cnt); c < cnt; c++) put(pos + c, fill, g);
        }
        if (rowm) {  // block-uniform
            __syncthreads();
            for (uint32_t i = t; i < min(tot, kStage); i += 256) {
                keys[s_base + i] = (K)st_key[i];
                vals[s_base + i] = st_val[i];
            }
        }
    }
    {
        // the large Gaussians: 256 bins of one Gaussian at a time, one per thread (its bin row's
        // spans, mask and open tiles), compacted by ballots, one reservation per round
        const uint32_t nbig = s_nbig;  // read after the barrier above (or the one at the top)
        const uint64_t lt = (1ull << lane) - 1ull;
        for (uint32_t j = 0; j < nbig; j++) {
            const uint32_t gb = s_big[j];
            const int rb = radii[gb];
            const float4 A = splats[gb].a;
            const float4 Bv = splats[gb].b;
            int bx0, by0, bx1, by1;
            tile_rect(A.x, A.y, rb, gx, gy, bx0, by0, bx1, by1);
            clip(bx0, by0, bx1, by1);  // non-empty: it was queued on the clipped rect
            float ccx, ccy, ccz;
            splat_conic(A, Bv, ccx, ccy, ccz);
            const CullEll eb = cull_setup(A.x, A.y, ccx, ccy, ccz, cull ? cull_qmax(Bv.w) : 0.f);
            const int Xs = bx0 >> 1, bw = ((bx1 + 1) >> 1) - Xs, Ys = by0 >> 1;
            const int nb = bw * (((by1 + 1) >> 1) - Ys);
            for (int b0 = 0; b0 < nb; b0 += 256) {
                const int b = b0 + t;
                uint32_t m = 0u;
                int X = 0, Y = 0;
                if (b < nb) {
                    Y = Ys + b / bw;
                    X = Xs + b % bw;
                    int l0, h0, l1, h1;
                    bin_row_spans(eb, cull, Y, bx0, bx1, by0, by1, l0, h0, l1, h1);
                    m = bin_mask(X, l0, h0, l1, h1);
                    if (m) m &= open4(X, Y);
                }
                const uint64_t bal = __ballot(m != 0u);
                __syncthreads();  // the previous round's reads of wsum / s_base are done
                if (lane == 0) wsum[w] = (uint32_t)__popcll(bal);
                __syncthreads();
                uint32_t bpre = 0, btot = 0;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    bpre += i < w ? wsum[i] : 0u;
                    btot += wsum[i];
                }
                if (btot == 0) continue;  // block-uniform
                if (t == 0) s_base = atomicAdd(n_total, btot);
                __syncthreads();
                if (m) {
                    const uint32_t pos = s_base + bpre + (uint32_t)__popcll(bal & lt);
                    keys[pos] = (K)(Y * bgx + X);
                    vals[pos] = gb | (m << BIN_SHIFT);
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_mark_visible(int P, const float* __restrict__ means3D,
                                                      const float* __restrict__ view, uint8_t* __restrict__ present) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const v3 pv = xform_point_4x3(load3(means3D + 3 * (size_t)i), view);
    present[i] = pv.z <= 0.2f ? 0 : 1;
}

// ---------------------------------------------------------------------------------------
// host launchers
static inline int blocks_for(long n, int b = 256) { return (int)((n + b - 1) / b); }

void launch_preprocess_views(const PreArgs& a, const PreViews& vs, hipStream_t st) {
    const int rows = a.n_out > a.P ? a.n_out : a.P;
    if (rows == 0 || vs.V <= 0) return;
    const dim3 grid(blocks_for(rows), vs.V);
    switch (a.colors_precomp ? 0 : a.D) {
        case 0: k_preprocess_views<0><<<grid, 256, 0, st>>>(a, vs); break;
        case 1: k_preprocess_views<1><<<grid, 256, 0, st>>>(a, vs); break;
        case 2: k_preprocess_views<2><<<grid, 256, 0, st>>>(a, vs); break;
        default: k_preprocess_views<3><<<grid, 256, 0, st>>>(a, vs); break;
    }
}

void launch_preprocess(const PreArgs& a, hipStream_t st) {
    const int rows = a.n_out > a.P ? a.n_out : a.P;
    if (rows == 0) return;
    const int nb = blocks_for(rows);
    // (staging the SH coefficients through LDS was measured slower: 1.68 vs 1.66 ms per step)
    switch (a.colors_precomp ? 0 : a.D) {
        case 0: k_preprocess<0><<<nb, 256, 0, st>>>(a); break;
        case 1: k_preprocess<1><<<nb, 256, 0, st>>>(a); break;
        case 2: k_preprocess<2><<<nb, 256, 0, st>>>(a); break;
        default: k_preprocess<3><<<nb, 256, 0, st>>>(a); break;
    }
}

template <typename K>
bool launch_duplicate(const DupArgs<K>& d, hipStream_t st) {
    if (d.P == 0 || d.nwin == 0 || d.win > (uint32_t)kSortMaxUnit) {  // win comes from radix_sort_plan
        if (d.zero && d.nzero > 0) (void)hipMemsetAsync(d.zero, 0, (size_t)d.nzero * sizeof(uint32_t), st);
        return false;
    }
    const bool second = d.first_b && d.nwin_b > 0 && d.win_b > 0 && d.win_b <= (uint32_t)kSortMaxUnit;
    if (!d.starts_done)
        k_window_starts<<<blocks_for(d.P), 256, 0, st>>>(d.n_list, d.off, d.pair0, d.win, d.nwin, d.first,
                                                         second ? d.n_list_b : d.n_list, second ? d.off_b : d.off,
                                                         d.pair0_b, second ? d.win_b : 1u, second ? d.nwin_b : 0,
                                                         d.first_b, d.zero, d.zero ? d.nzero : 0);
    auto kern = d.open_bits ? k_duplicate<K, true> : k_duplicate<K, false>;
    const bool ord = d.open_bits && d.order_out && d.order_cost && d.order_flag && d.order_T > 0;
    kern<<<d.nwin + (ord ? 1 : 0), 256, 0, st>>>(d.n_list, d.idx, d.off, d.splats, d.radii, d.gx, d.gy, d.cull,
                                                  d.first, d.pair0, d.win, d.L_dev, d.keys, d.vals, d.dbits, d.counts,
                                                  d.nwin, d.open_bits, d.unit_len, d.n_total, ord ? d.order_cost : nullptr,
                                                  ord ? d.order_out : nullptr, d.order_flag, d.order_T);
    return !d.starts_done && second;
}
template bool launch_duplicate<uint16_t>(const DupArgs<uint16_t>&, hipStream_t);
template bool launch_duplicate<uint32_t>(const DupArgs<uint32_t>&, hipStream_t);

template <typename K>
void launch_dup_gather(const DupArgs<K>& d, hipStream_t st) {
    if (d.P == 0) return;
    const bool ord = d.order_out && d.order_cost && d.order_flag && d.order_T > 0;
    const Tuning& tu = tuning();
    k_dup_gather<K><<<blocks_for(d.P) + (ord ? 1 : 0), 256, 0, st>>>(
        d.tiles, d.splats, d.radii, d.gx, d.gy, d.cull, d.keys, d.vals, d.open_bits, d.n_total,
        ord ? d.order_cost : nullptr, ord ? d.order_out : nullptr, d.order_flag, d.order_T, d.n_list, d.idx,
        tu.dup_big_bins, tu.dup_b_rows ? 1 : 0, d.gather_mark);
}
template void launch_dup_gather<uint16_t>(const DupArgs<uint16_t>&, hipStream_t);
template void launch_dup_gather<uint32_t>(const DupArgs<uint32_t>&, hipStream_t);

void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t st) {
    if (P == 0) return;
    k_mark_visible<<<blocks_for(P), 256, 0, st>>>(P, means3D, view, present);
}

}  // namespace rr
