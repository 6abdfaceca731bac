// rr_sort.hip — stable LSD radix sort of (key, u32 value) pairs, written for CDNA4.
//
// Used for the per-frame depth sort (P keys, 32 bits) and the tile sort (L pairs, <= 16 bits);
// replaces rocPRIM's device radix sort (Onesweep look-back latency bound here; merge path below
// 2^20 items).
//
// Each pass sorts by one digit of <= 8 bits with a count / scan / scatter split over "units" of
// one workgroup (4 wave64s) x R rounds x 64 items (R chosen per call so that small inputs still
// spread over enough workgroups):
//   * k_rs_count: digit histogram of the unit in LDS -> counts[digit][unit] (digit-major);
//   * rocprim::exclusive_scan over counts gives every (digit, unit) its first output slot;
//   * k_rs_scatter: (1) per-wave digit counts, (2) block-local digit starts in LDS, (3) each wave
//     walks its rounds in order; lanes holding the same digit find each other with one ballot per
//     digit bit (wave-wide match), rank = popcount of lower matching lanes, the group leader
//     advances the per-(wave, digit) cursor; the item is staged in LDS at its block-local sorted
//     position, (4) the staged unit is written out in order, so consecutive threads write
//     consecutive addresses of each digit's run (coalesced) instead of scattering single items.
// Order inside a unit is (wave, round, lane) = input order and units are scanned in order, so
// every pass is stable.  Passes = ceil(bits / 8) with the bits spread evenly (13 -> 7 + 6).
#include <rocprim/device/device_scan.hpp>

#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

namespace {

constexpr int kWaves = 4;       // waves per workgroup (unit)
constexpr int kMaxRounds = 16;  // rounds of 64 items per wave
constexpr int kMaxUnitItems = 64 * kWaves * kMaxRounds;  // 4096
static_assert(kMaxUnitItems == kSortMaxUnit, "rr_kernels.hpp kSortMaxUnit");

template <typename K>
__global__ __launch_bounds__(64 * kWaves) void k_rs_count(const K* __restrict__ keys, size_t n, int shift, int dbits,
                                                          int rounds, uint32_t* __restrict__ counts, int units) {
    __shared__ uint32_t hist[256];
    const int t = threadIdx.x;
    const int ndig = 1 << dbits;
    for (int d = t; d < ndig; d += 64 * kWaves) hist[d] = 0;
    const int unit = blockIdx.x;
    const size_t base = (size_t)unit * rounds * 64 * kWaves;
    const uint32_t mask = (uint32_t)ndig - 1u;
    uint32_t dr[kMaxRounds];
#pragma unroll
    for (int r = 0; r < kMaxRounds; r++) {  // all loads in flight before the first LDS atomic
        const size_t i = base + (size_t)r * 64 * kWaves + t;
        dr[r] = (r < rounds && i < n) ? (((uint32_t)keys[i] >> shift) & mask) : 0xffffffffu;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kMaxRounds; r++)
        if (dr[r] != 0xffffffffu) atomicAdd(&hist[dr[r]], 1u);
    __syncthreads();
    for (int d = t; d < ndig; d += 64 * kWaves) counts[(size_t)d * units + unit] = hist[d];
}

template <typename K>
__global__ __launch_bounds__(64 * kWaves) void k_rs_scatter(const K* __restrict__ keys_in,
                                                            const uint32_t* __restrict__ vals_in,
                                                            K* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
                                                            size_t n, int shift, int dbits, int rounds,
                                                            const uint32_t* __restrict__ offsets, int units) {
    __shared__ uint32_t wcnt[kWaves][256];  // per-wave digit counts, then per-wave cursors
    __shared__ uint32_t dstart[256];        // block-local start of each digit's run
    __shared__ uint32_t goff[256];          // global slot of block-local position 0 of each digit's run
    __shared__ uint32_t s_val[kMaxUnitItems];
    __shared__ K s_key[kMaxUnitItems];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int ndig = 1 << dbits;
    const uint32_t mask = (uint32_t)ndig - 1u;
    const int unit = blockIdx.x;
    const size_t ubase = (size_t)unit * rounds * 64 * kWaves;
    // wave w owns the contiguous items [wbase, wbase + 64 * rounds) of the unit
    const size_t wbase = ubase + (size_t)w * 64 * rounds;
    for (int d = lane; d < ndig; d += 64) wcnt[w][d] = 0;
    for (int d = t; d < ndig; d += 64 * kWaves) goff[d] = offsets[(size_t)d * units + unit];
    // the wave's items go to registers once (all loads in flight together); counting, ranking
    // and staging then run from registers
    K kr[kMaxRounds];
    uint32_t vr[kMaxRounds];
#pragma unroll
    for (int r = 0; r < kMaxRounds; r++) {
        const size_t i = wbase + (size_t)r * 64 + lane;
        const bool valid = r < rounds && i < n;
        kr[r] = valid ? keys_in[i] : (K)0;
        vr[r] = valid ? (vals_in ? vals_in[i] : (uint32_t)i) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kMaxRounds; r++) {
        const size_t i = wbase + (size_t)r * 64 + lane;
        if (r < rounds && i < n) atomicAdd(&wcnt[w][((uint32_t)kr[r] >> shift) & mask], 1u);
    }
    __syncthreads();
    // block-local starts: digits in order, then waves in order inside each digit.  Wave 0 scans the
    // <= 256 digit totals: 4 consecutive digits per lane, then a 6-step shuffle scan of lane sums.
    if (w == 0) {
        uint32_t tot[4], sum = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int d = 4 * lane + i;
            tot[i] = 0;
            if (d < ndig)
#pragma unroll
                for (int v = 0; v < kWaves; v++) tot[i] += wcnt[v][d];
            sum += tot[i];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += y;
        }
        uint32_t run = incl - sum;  // exclusive prefix of this lane's first digit
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int d = 4 * lane + i;
            if (d < ndig) {
                dstart[d] = run;
                goff[d] -= run;
                uint32_t r2 = run;
#pragma unroll
                for (int v = 0; v < kWaves; v++) {
                    const uint32_t x = wcnt[v][d];
                    wcnt[v][d] = r2;
                    r2 += x;
                }
            }
            run += tot[i];
        }
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < kMaxRounds; r++) {
        if (r >= rounds || wbase + (size_t)r * 64 >= n) continue;  // wave-uniform; keeps the loop unrollable
        const size_t i = wbase + (size_t)r * 64 + lane;
        const bool valid = i < n;
        const K k = kr[r];
        const uint32_t v = vr[r];
        const uint32_t d = ((uint32_t)k >> shift) & mask;
        uint64_t m = __ballot(valid);
        for (int b = 0; b < dbits; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(m & lt);
        const uint32_t lpos = wcnt[w][d] + rank;  // every lane reads before any leader writes
        __builtin_amdgcn_wave_barrier();
        if (valid && rank == 0) wcnt[w][d] = lpos + (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
        if (valid) {
            s_key[lpos] = k;
            s_val[lpos] = v;
        }
    }
    __syncthreads();
    const int nu = (int)min((size_t)rounds * 64 * kWaves, n - ubase);
    for (int j = t; j < nu; j += 64 * kWaves) {
        const K k = s_key[j];
        const uint32_t d = ((uint32_t)k >> shift) & mask;
        const uint32_t pos = goff[d] + (uint32_t)j;
        if (keys_out) keys_out[pos] = k;
        vals_out[pos] = s_val[j];
    }
}

struct SortLayout {
    void* keys_alt;
    uint32_t* vals_alt;
    uint32_t* counts;
    uint32_t* offsets;
    void* scan_temp;
    size_t scan_bytes;
    size_t total;
};

// rounds per wave: full 16 for large inputs, fewer for small ones so that there are >= ~1024 units
int rounds_for(size_t n) {
    int r = kMaxRounds;
    while (r > 1 && (n + (size_t)64 * kWaves * r - 1) / ((size_t)64 * kWaves * r) < 1024) r >>= 1;
    return r;
}

template <typename K>
SortLayout sort_layout(void* buf, size_t n, int bits) {
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    SortLayout s{};
    const int rounds = rounds_for(n);
    const size_t units = (n + (size_t)64 * kWaves * rounds - 1) / ((size_t)64 * kWaves * rounds);
    const int passes = bits <= 0 ? 0 : (bits + 7) / 8;
    const int dmax = passes ? (bits + passes - 1) / passes : 0;
    const size_t nc = std::max<size_t>(((size_t)1 << dmax) * units, 1);
    s.scan_bytes = 0;
    if (n > 0)
        (void)rocprim::exclusive_scan(nullptr, s.scan_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, nc,
                                      rocprim::plus<uint32_t>(), (hipStream_t)0);
    char* p = static_cast<char*>(buf);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        void* r = p ? p + off : nullptr;
        off = al(off + std::max<size_t>(bytes, 1));
        return r;
    };
    s.keys_alt = take(n * sizeof(K));
    s.vals_alt = static_cast<uint32_t*>(take(n * 4));
    s.counts = static_cast<uint32_t*>(take(nc * 4));
    s.offsets = static_cast<uint32_t*>(take(nc * 4));
    s.scan_temp = take(s.scan_bytes);
    s.total = off;
    return s;
}

}  // namespace

template <typename K>
size_t radix_sort_temp_bytes(size_t n, int bits) {
    return sort_layout<K>(nullptr, n, bits).total;
}

template <typename K>
RadixPlan radix_sort_plan(void* temp, size_t n, int begin_bit, int end_bit) {
    RadixPlan p{};
    const int bits = end_bit - begin_bit;
    if (n == 0 || bits <= 0) return p;
    const SortLayout s = sort_layout<K>(temp, n, bits);
    const int passes = (bits + 7) / 8;
    p.rounds = rounds_for(n);
    p.unit_items = 64 * kWaves * p.rounds;
    p.units = (int)((n + p.unit_items - 1) / p.unit_items);
    p.dbits0 = (bits + passes - 1) / passes;
    p.counts = s.counts;
    return p;
}

template <typename K>
hipError_t radix_sort_pairs(void* temp, size_t temp_bytes, const K* keys_in, K* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, size_t n, int begin_bit, int end_bit, hipStream_t st,
                            bool first_counts_ready) {
    const int bits = end_bit - begin_bit;
    if (n == 0) return hipSuccess;
    if (n > 0xffffffffull || bits <= 0 || bits > (int)(8 * sizeof(K))) return hipErrorInvalidValue;
    const SortLayout s = sort_layout<K>(temp, n, bits);
    if (temp_bytes < s.total) return hipErrorInvalidValue;
    const int passes = (bits + 7) / 8;
    const int rounds = rounds_for(n);
    const int units = (int)((n + (size_t)64 * kWaves * rounds - 1) / ((size_t)64 * kWaves * rounds));
    const K* ksrc = keys_in;
    const uint32_t* vsrc = vals_in;
    int shift = begin_bit;
    for (int p = 0; p < passes; p++) {
        // spread the bits evenly over the passes (13 -> 7 + 6)
        const int dbits = (bits - (shift - begin_bit) + (passes - p) - 1) / (passes - p);
        const bool last = p == passes - 1;
        // destinations alternate so that the last pass lands in the caller's buffers
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        K* kdst = to_out ? keys_out : static_cast<K*>(s.keys_alt);
        uint32_t* vdst = to_out ? vals_out : s.vals_alt;
        if (!last && kdst == nullptr) return hipErrorInvalidValue;  // intermediate passes need key storage
        const size_t nc = ((size_t)1 << dbits) * (size_t)units;
        if (!(p == 0 && first_counts_ready))
            k_rs_count<K><<<units, 64 * kWaves, 0, st>>>(ksrc, n, shift, dbits, rounds, s.counts, units);
        size_t sb = s.scan_bytes;
        hipError_t e = rocprim::exclusive_scan(s.scan_temp, sb, s.counts, s.offsets, 0u, nc,
                                               rocprim::plus<uint32_t>(), st);
        if (e != hipSuccess) return e;
        k_rs_scatter<K><<<units, 64 * kWaves, 0, st>>>(ksrc, vsrc, kdst, vdst, n, shift, dbits, rounds, s.offsets,
                                                       units);
        ksrc = kdst;
        vsrc = vdst;
        shift += dbits;
    }
    return hipGetLastError();
}

template size_t radix_sort_temp_bytes<uint16_t>(size_t, int);
template size_t radix_sort_temp_bytes<uint32_t>(size_t, int);
template hipError_t radix_sort_pairs<uint16_t>(void*, size_t, const uint16_t*, uint16_t*, const uint32_t*, uint32_t*,
                                               size_t, int, int, hipStream_t, bool);
template hipError_t radix_sort_pairs<uint32_t>(void*, size_t, const uint32_t*, uint32_t*, const uint32_t*, uint32_t*,
                                               size_t, int, int, hipStream_t, bool);
template RadixPlan radix_sort_plan<uint16_t>(void*, size_t, int, int);
template RadixPlan radix_sort_plan<uint32_t>(void*, size_t, int, int);

}  // namespace rr
