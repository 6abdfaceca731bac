// rr_kernels.hpp — kernel argument blocks and host launchers shared by the .hip units.
#pragma once
#include "rr_common.hpp"
#include "../../include/rain_raster.h"

namespace rr {

// Per-frame scalars of the depth-sort-free binning (rr_bin.hip), in the geometry buffer: written by
// the split scan's first launch (L, rect, wide, cut; it also copies L, rect and wide to the host
// mailbox) and by the split scan's last thread (LA, LB, GA, GB: read on the device only).  Also the device copy the
// no-mailbox read-back path reads.
struct FrameTotals {
    unsigned long long L;     // (bin, Gaussian) pairs of the frame
    unsigned long long rect;  // bounding-rect tiles (the reference's num_rendered)
    uint32_t cut;             // early-stop split: phase A = Gaussians with depth key < cut
    uint32_t wide;            // a visible depth key needs more than kDepthKeyBits bits
    uint32_t LA, LB;          // pairs of phase A / phase B (saturated to 32 bits)
    uint32_t GA, GB;          // Gaussians of phase A / phase B (lengths of the PhaseLists)
};
// The two phases' Gaussian lists in index order (rr_bin.hip launch_split_scan): entry r of a phase
// is its r-th Gaussian's index and the inclusive sum of the phase's pairs up to it.
struct PhaseLists {
    uint32_t* idx_a;
    uint32_t* off_a;
    uint32_t* idx_b;
    uint32_t* off_b;
    // first entry of every window of kSplitWin consecutive pairs of the phase's list (window k starts
    // inside entry first[k]'s pair range), for the first nwin windows: the windowed duplicate's
    // starts, marked by the split scan when the bin sort's unit is kSplitWin pairs
    uint32_t* first_a;
    uint32_t* first_b;
    uint32_t nwin;
};
constexpr uint32_t kSplitWin = 2048;

struct PreArgs {
    int P, D, M, W, H, gx, gy, prefiltered;
    float tanfovx, tanfovy, focal_x, focal_y, scale_modifier, low_pass;
    const float* means3D;
    const float* shs;
    const float* colors_precomp;
    const float* opacities;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    const float* view;
    const float* proj;
    const float* campos;
    int* radii;
    Splat* splats;
    uint2* tiles;                // {pairs this Gaussian emits (after culling), bounding-rect tile count}
    uint32_t* depth_keys;
    int cull;                    // exact tile culling on/off
    int raw;                     // RR_FLAG_RAW_PARAMS: apply the GaussianModel getters in-kernel
    const float* shs_rest;       // raw mode: f_rest [P,M-1,3] (shs = f_dc [P,1,3])
    float4* normals;             // RR_FLAG_AUX_NORMAL: view-space unit normal per visible Gaussian, else null
    uint2* block_sums;           // optional [ceil(P/256)]: per-block sums of tiles[] (pairs, rect tiles)
    uint32_t* block_wide;        // with block_sums: per block, 1 if a visible depth key needs > kDepthKeyBits
    int n_out;                   // rows written (>= P): rows P..n_out-1 get the culled outputs (radius 0,
                                 // no pairs, the largest depth key) — the padding rows of a row block
    float* wire;                 // optional (the sharded step's send chunks): per row the 10-float
                                 // wire record (splat_to_wire) instead of splats[] and depth_keys[]
};

// The sharded step's wire record of a splat: the 10 floats Splat holds that cannot be recomputed
// (x, y, qa, qb, qc, depth, o, r, g, b); log2 o, 1/o and the depth key are rebuilt by the
// receiver with the preprocess's own expressions (splat_derived), so the unpacked geometry is
// bitwise the preprocess's.
__device__ __forceinline__ void splat_derived(float o, float& log2o, float& inv_o) {
    log2o = __builtin_amdgcn_logf(o);
    inv_o = o > 0.f ? 1.0f / o : 0.f;
}
constexpr int kWireFloats = 10;
void launch_unpack_rows(int world, int rows_per_rank, const char* recv, size_t chunk_bytes,
                        const size_t field_offsets[5], Splat* splats, uint2* tiles, uint32_t* depth_keys, int* radii,
                        uint2* block_sums, uint32_t* block_wide, hipStream_t st);

// Depth keys: the float bits of the view depth minus those of the smallest float above the near
// plane (0.2f = 0x3E4CCCCD), so the keys of depths up to ~13107 fit 27 bits and the depth sort runs
// 3 passes; a frame with a deeper visible Gaussian is re-sorted on all 32 bits (the preprocess
// flags it, the host reads the flag with the pair counts).  Culled Gaussians keep 0xffffffff,
// whose low 27 bits are the maximum: they still sort behind every visible one, and their own order
// is irrelevant (no pairs).
constexpr uint32_t kDepthKeyBase = 0x3E4CCCCEu;
constexpr int kDepthKeyBits = 27;

// Early-stop binning (rr_api.hip): the tile lists are built in two phases.  Phase A bins the
// depth-ordered pairs [0, L_A) for every tile and blends them; a tile whose pixels have all
// saturated is final.  Phase B bins the pairs [L_A, L) only for the tiles still open and resumes
// their blend from the state phase A left in the image buffers.  A tile's list is then
// A-list ++ B-list (ranges / ranges_b), which is exactly the prefix of its full depth-ordered
// list that blending can reach.
enum BlendPhase { kBlendSingle = 0, kBlendPhaseA = 1, kBlendPhaseB = 2 };
constexpr uint32_t kDoneBit = 0x80000000u;  // n_contrib between the phases: pixel saturated

struct BlendFwdArgs {
    int W, H, gx, gy;
    const uint2* ranges;
    const uint32_t* point_list;
    const Splat* splats;
    const float* bg;
    float* final_T;
    uint32_t* n_contrib;
    uint32_t* tile_max;
    float* out_color;
    float* out_depth;
    const uint2* ranges_b;  // phase B lists
    uint8_t* open;          // [T] tile still open after phase A
    uint32_t* open_bits;    // [ceil(T/32)] the same as a bitmask (cleared with the ranges; phase A ORs)
    int phase;              // BlendPhase
    const float4* normals;  // aux normal output (RR_FLAG_AUX_NORMAL): per-Gaussian normals and
    float* out_normal;      // the blended normal map [3,H,W]; both null otherwise
    uint32_t* trace;        // RR_FWD_TRACE builds only: per-wave timing records (rr_debug_set_fwd_trace)
    // the backward's accumulator workspace (rr_set_forward_workspace), zero-filled by extra
    // workgroups after the tiles' (dispatched last: they run in the blend's drain); null: none
    float4* clear;
    size_t clear_n4;
};

struct BlendBwdArgs {
    int W, H, gx, gy;
    const uint2* ranges;
    const uint2* ranges_b;  // phase-B lists (all {0,0} for single-phase binning)
    const uint32_t* point_list;
    const Splat* splats;
    const uint32_t* tile_max;
    const float* final_T;
    const uint32_t* n_contrib;
    const float* bg;
    const float* dL_dpix;
    float* gacc;      // [P][GACC_STRIDE]
    uint32_t* order;  // [T] scratch: tile of each workgroup, heaviest first (k_tile_order); null: XCD order
};

struct GaussBwdArgs {
    int P, D, M;
    float tanfovx, tanfovy, focal_x, focal_y, scale_modifier, low_pass;
    const float* means3D;
    const float* shs;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    const float* view;
    const float* proj;
    const float* campos;
    const int* radii;
    const float* gacc;
    float* dL_dmeans2D;
    float* dL_dcolors;
    float* dL_dopacity;
    float* dL_dmeans3D;
    float* dL_dcov3D;
    float* dL_dsh;
    float* dL_dscales;
    float* dL_drot;
    int raw;
    const float* opacities;  // raw mode: logits (sigmoid backward)
    const float* shs_rest;
    float* dL_dsh_rest;
    float* grad_accum;
    float* denom;
    float* max_radii2D;
    // fused optimizer step (raw mode): copied BY VALUE into the kernel arguments (the caller's
    // rr_adam lives in host memory); use_adam says whether it is valid
    rr_adam adam;
    int use_adam;
    // with use_adam: the next frame's preprocess on the stepped parameters (rr_next_frame): its
    // camera, frame values and output arrays (geometry buffer, radii); has_next says whether valid
    PreArgs next;
    int has_next;
};

void launch_preprocess(const PreArgs& a, hipStream_t st);
// One launch preprocessing the same rows for up to kMaxPreViews views (the Gaussian-sharded step's
// owner preprocess): view v = blockIdx.y takes its camera from vs.v[v] and writes every output
// array of PreArgs displaced by v * vs.stride bytes.
constexpr int kMaxPreViews = 16;
struct PreView {
    const float* view;
    const float* proj;
    const float* campos;
    float tanfovx, tanfovy, focal_x, focal_y, low_pass;
    int W, H, gx, gy;
};
struct PreViews {
    PreView v[kMaxPreViews];
    size_t stride;
    int V;
};
void launch_preprocess_views(const PreArgs& a, const PreViews& vs, hipStream_t st);
// The pair-count scan (rasterizer_impl.cu:269; rr_bin.hip launch_split_scan) in blocks of
// kPairScanItems: per-block totals, then each block scans its items on top of the sum of the earlier
// totals: up to kPairScanDirectBlocks blocks (P <= 1,048,576) every block sums those totals itself
// (2 launches), above it one workgroup scans them first (3 launches; Tuning::pair_scan_direct_blocks
// moves the cut-over, tests force both paths).
constexpr int kPairScanItems = 2048;                 // items per block (256 threads x 8)
constexpr int kPairScanDirectBlocks = 512;
// rr_bin.hip: the depth-sort-free binning
// The phases' Gaussian lists (PhaseLists, ft->GA / GB entries) and, computed by every workgroup of
// its first launch, the frame's totals and early-stop depth cut (published to the host mailbox);
// the last thread leaves {LA, LB, GA, GB} in ft.  temp: split_scan_temp_bytes(P)
size_t split_scan_temp_bytes(int P);
struct CutArgs {
    const uint2* block_sums;
    const uint32_t* block_wide;
    uint32_t den, min_pairs;
    uint32_t* box;  // host mailbox (may be null) and this read's sequence number
    uint32_t seq;
};
void launch_split_scan(const uint2* tiles, const uint32_t* keys, int P, PhaseLists lists, FrameTotals* ft, void* temp,
                       int direct_blocks, uint32_t* zero, int nzero, const CutArgs& cut,
                       hipStream_t st);  // zero (optional): nzero words cleared by its first launch
// Per bin: the depth order of its run of the bin-sorted pairs and its four tiles' lists (bounds:
// the bins' runs, from the bin sort's last scatter).  Runs longer than the LDS cap are sorted in
// their own point_list region and written back over vals.
template <typename K>
void launch_sortexpand(const K* keys, const uint32_t* vals, const uint32_t* depth_keys, const FrameTotals* ft, int gx,
                       int gy, uint32_t out_base, uint32_t* point_list, uint2* ranges, const uint32_t* open_bits,
                       const uint2* bounds, hipStream_t st);
// Phase B of the gather path (rr_bin.hip k_bin_count + k_bin_scatter + k_sortexpand): the densely
// emitted, unordered phase-B pairs (k_dup_gather) counted per bin (bin_cnt, zero on entry) and
// dropped into their bins' runs — no bin sort.  kept: receives the pairs the bins hold.  false:
// more bins than one workgroup scans (nothing launched).
template <typename K>
bool launch_sortexpand_small(int P, const K* keys, const uint32_t* vals, const uint32_t* n_dev, uint32_t* bin_cnt,
                             uint32_t* vals_sorted, const uint32_t* depth_keys, const FrameTotals* ft, int gx, int gy,
                             uint32_t out_base, uint32_t* point_list, uint2* ranges, const uint32_t* open_bits,
                             uint2* bounds, uint32_t* kept, hipStream_t st);
template <typename K>
struct DupArgs {
    int P;                       // capacity of the lists (the frame's Gaussians)
    const uint32_t* n_list;      // device: entries of the phase's list (FrameTotals GA / GB)
    const uint32_t* idx;         // the phase's Gaussians in index order (PhaseLists)
    const uint32_t* off;         // their inclusive pair offsets
    const Splat* splats;
    const int* radii;
    int gx, gy, cull;
    uint32_t* first;     // [nwin] first Gaussian of each window
    uint32_t pair0;      // pair index of window 0
    uint32_t win;        // pairs per window (= sort unit)
    int nwin;
    const uint32_t* L_dev;  // device: end of the pair range (FrameTotals LA / LB)
    K* keys;             // window k writes [k*win, ...)
    uint32_t* vals;
    int dbits;           // first-pass digit width of the tile sort
    uint32_t* counts;    // its per-window digit counts
    // phase B (early-stop binning); all null for an unfiltered pass
    const uint32_t* open_bits;
    uint32_t* unit_len;
    uint32_t* n_total;
    // optional (phase B): one extra workgroup computes the backward blend's tile order from the
    // phase-A tile_max (order_cost) into order_out and sets *order_flag = order_T, so that the
    // backward prologue skips its own one-workgroup sort (its critical path)
    const uint32_t* order_cost;
    uint32_t* order_out;
    uint32_t* order_flag;
    int order_T;
    // optional: words cleared by the window-starts kernel before the duplicate runs (the frame's
    // tile ranges and counters; saves a memset launch on the path right after the pair-count
    // readback)
    uint32_t* zero;
    int nzero;
    // optional second window set (the phase-B windows over the phase-B list, computed in the
    // phase-A launch of the window-starts kernel: one launch less on the path); starts_done: this
    // pass's windows were computed that way, skip the kernel
    uint32_t* first_b;
    uint32_t pair0_b, win_b;
    int nwin_b;
    const uint32_t* n_list_b;
    const uint32_t* off_b;
    bool starts_done;
    // the gather path (launch_dup_gather): every Gaussian's {pairs, rect tiles}; n_total receives
    // the phase's reserved slots (zero on entry)
    const uint2* tiles;
    uint32_t* gather_mark;  // set to 1 by the gather path (the frame statistics read which path ran)
};
// returns whether the window starts (both sets) were computed
template <typename K>
bool launch_duplicate(const DupArgs<K>& d, hipStream_t st);
// phase B by the gather path: one thread per entry of the split scan's phase-B list (d.idx, with
// d.n_list entries), its pairs on open tiles written densely and unordered at d.keys / d.vals,
// the slots reserved added to *d.n_total (rr_forward.hip k_dup_gather)
template <typename K>
void launch_dup_gather(const DupArgs<K>& d, hipStream_t st);
void launch_blend_fwd(const BlendFwdArgs& a, hipStream_t st);
void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t st);

void launch_blend_bwd(const BlendBwdArgs& a, hipStream_t st);  // a.order: from launch_bwd_prologue
// clears the nfloats gradient accumulators and, with order, writes the backward's tile order
// order_flag (may be null): *order_flag == T means the order was already computed this frame
void launch_bwd_prologue(float* gacc, size_t nfloats, int T, const uint32_t* tile_max, uint32_t* order,
                         const uint32_t* order_flag,
                         hipStream_t st);

// Largest sort unit (items per workgroup) of rr_sort.hip; the duplicate kernel's LDS windows are
// sort units, so it sizes its staging arrays with this too.
constexpr int kSortMaxUnit = 4096;
// point_list is followed by at least this many readable u32 (the scalar-record forward blend loads
// the ids of a whole group, up to 8, before masking the ones past its list's end)
constexpr int kPointListPad = 16;

// rr_sort.hip: stable LSD radix sort of (K key, u32 value) pairs on bits [begin_bit, end_bit).
// vals_in == nullptr means values = input index.  keys_out may be nullptr only for a single pass.
// n is the (host-known) capacity; unit_len (per-unit item counts of a sparse first pass, counts
// produced by the caller) and n_dev (device-side item count after compaction) are optional.
// n_hint (0: n) is the expected count the unit length is chosen for when n is only a capacity
// (units then cover n; those past the device count are empty).
template <typename K>
size_t radix_sort_temp_bytes(size_t n, int bits, size_t n_hint = 0);
template <typename K>
hipError_t radix_sort_pairs(void* temp, size_t temp_bytes, const K* keys_in, K* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, size_t n, int begin_bit, int end_bit, hipStream_t st,
                            bool first_counts_ready = false, const uint32_t* unit_len = nullptr,
                            const uint32_t* n_dev = nullptr, size_t n_hint = 0, uint2* bounds = nullptr);
// bounds (optional, [1 << (end_bit - begin_bit)], zero on entry): each key's run in the sorted output,
// encoded {~start, end} (a key without items keeps {0, 0}; rr_bin.hip k_sortexpand decodes), written by
// the last pass's scatter
const char* radix_sort_last_error();  // which check failed in the last radix_sort_pairs call
// Unit geometry of a sort and where its first-pass digit counts live, so that a producer kernel
// can emit counts[digit * units + unit] for the lowest dbits0 bits itself (then pass
// first_counts_ready = true).
struct RadixPlan {
    uint32_t* counts;
    int units, unit_items, rounds, dbits0;
};
template <typename K>
RadixPlan radix_sort_plan(void* temp, size_t n, int begin_bit, int end_bit, size_t n_hint = 0);
void launch_gauss_bwd(const GaussBwdArgs& a, hipStream_t st);
// The Gaussian-sharded multi-GPU step (rr_gauss_backward_views): one view's camera as the
// per-Gaussian backward reads it.
struct ViewCam {
    const float* view;
    const float* proj;
    const float* campos;
    float tanfovx, tanfovy, focal_x, focal_y, low_pass;
};
// rows a.P of a row block, V <= 16 views (records [V][rec_rows][10]); returns 1 on a bad V
int launch_gauss_bwd_views(const GaussBwdArgs& a, const ViewCam* cams, int V, const float* records, int rec_rows,
                           float grad_scale, hipStream_t st);
void launch_pack_records(const float* gacc, const int* radii, int P, int Q, int chunk_rows, float* rec,
                         hipStream_t st);

}  // namespace rr

namespace rr {
// Runtime tuning (include/rain_raster.h rr_set_tuning / rr_set_binning_config): the early-stop
// split, and knobs that force a product path of larger frames or scenes onto the small frames of
// the tests (every setting gives the same lists, images and gradients).  One record per HIP device
// (the device current at the call; rr_api.hip tuning()), so that a process driving several GPUs
// does not share them across devices.
constexpr int kMaxDevices = 64;
struct Tuning {
    uint32_t early_den = 3;          // early-stop split: phase A holds ~1/early_den of the pairs
    uint32_t early_min = 1u << 16;   // frames below this many pairs are binned in one phase
    int pair_scan_direct_blocks = kPairScanDirectBlocks;  // 3-launch pair-count scan above it
    bool wide_bin_keys = false;      // 32-bit bin keys (frames of > 65536 bins)
    bool b_gather = true;            // phase B by the gather path (false: the windowed path of > 16384 bins)
    bool dup_b_rows = true;          // phase-B gather: row masks (false: the flat mask of > 128 tiles wide)
    int dup_big_bins = 32;           // phase-B gather: Gaussians over this many bins emitted per workgroup
    bool sx_bucket = true;           // per-bin order by the bucket sort (false: LSD passes only)
    int sx_lds_cap = 0;              // per-bin runs over this many pairs through the global path (0: LDS cap)
    int sort_min_units = 128;        // radix sorts: target unit count
    int sort_min_units_tile = 1024;  // the same for the bin sorts (<= 16-bit keys)
    int sort_max_rounds = 16;        // cap on 64-item rounds per wave in a sort unit
};
Tuning& tuning();  // the current device's
void set_fwd_trace(void* dev_buf);
}  // namespace rr
