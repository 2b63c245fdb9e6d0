// cc_engine.hip — the ConsensusCruncher consensus hot path on MI355X (gfx950).
//
// One HIP stream per context; every stage is a chain of data-parallel kernels
// over struct-of-arrays records resident in HBM.  The reference's sequential
// dictionary program (consensus_helper.read_bam, consensus_helper.py:308-506,
// and the stage loops of SSCS_maker.py:272-346, DCS_maker.py:210-282,
// singleton_correction.py:209-319) is restated as sort/scan/segment steps:
//
//   read_bam    k_classify   filters of consensus_helper.py:404-420 + counters
//               radix sort   (qname hash, stream pos)      -> pair_dict by qname (:426-432)
//               k_pair_mark  runs of equal qname -> pairs completed at the 2nd mate
//               k_pair_keys  which_read/which_strand/cigar_order/sscs_qname/unique_tag (:57-305)
//               radix sort   (tag hash, read-end index)     -> read_dict / tag_dict (:455-494)
//               k_fam_*      families, members in completion order, "line read twice" drop
//               radix sort   (consensus-tag hash, creation) -> csn_pair_dict (:469-489)
//   SSCS        k_sscs_vote_swar consensus_maker (SSCS_maker.py:81-168) fused with read_mode /
//                            consensus_flag (consensus_helper.py:509-565)
//   DCS         k_dcs_decide duplex_tag hash-join + the duplex_dict rule (DCS_maker.py:245-282)
//   SC          k_sc_decide  SSCS-first then singleton lookup (singleton_correction.py:278-319)
//               k_duplex_vote_swar duplex_consensus (DCS_maker.py:99-123 / singleton_correction.py:61-86)
//
// All keys are exact: 64-bit hashes only order the sorts; equal-hash neighbours are
// always compared field by field and a collision aborts with CC_E_COLLISION so the
// caller re-runs with a new seed.
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include <dlfcn.h>
#include <sched.h>

#include <chrono>

#include <hip/hip_runtime.h>
#include <atomic>
#include <rocprim/rocprim.hpp>
#include <map>
#include <memory>
#include <type_traits>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/consensuscruncher_amd.h"

// every device operation this library enqueues is counted (cc_launch_count: the bench's launches
// per step): kernel launches, memsets, async copies, and each rocPRIM call once
static std::atomic<long long> g_launches{0};
#undef hipLaunchKernelGGL
#define hipLaunchKernelGGL(kernelName, ...)                                                          \
    do {                                                                                            \
        g_launches.fetch_add(1, std::memory_order_relaxed);                                         \
        hipLaunchKernelGGLInternal((kernelName), __VA_ARGS__);                                      \
    } while (0)
#define hipMemsetAsync(...) (g_launches.fetch_add(1, std::memory_order_relaxed), ::hipMemsetAsync(__VA_ARGS__))
#define hipMemcpyAsync(...) (g_launches.fetch_add(1, std::memory_order_relaxed), ::hipMemcpyAsync(__VA_ARGS__))

// ------------------------------------------------------------------ error bits (device)
enum : uint32_t {
    EB_COLLISION = 1u << 0,
    EB_DUP_QNAME = 1u << 1,
    EB_AMBIGUOUS = 1u << 2,
    EB_N_HIGHQ = 1u << 3,
    EB_BAD_BASE = 1u << 4,
    EB_SHORT = 1u << 5,
    EB_NO_QUAL = 1u << 6,
    EB_NO_CIGAR = 1u << 7,
    EB_RG = 1u << 8,
    EB_THR = 1u << 9,
    EB_TOO_LONG = 1u << 10,   // k_table_cols: a length beyond the 16-bit member-record fields
    EB_KEYERROR = 1u << 12,   // the reference raises KeyError here (DCS_maker.py:258)
    EB_CHAIN = 1u << 13,      // a duplex chain longer than DUPLEX_CHAIN
    EB_NEEDSORT = 1u << 14,   // coordinate pairing met a qname seen more than twice: re-run on the sort path
    EB_PLAN = 1u << 11,       // a planned capacity was exceeded (the pass re-runs exactly)
    EB_DEEPSORT = 1u << 15,   // a deep family out of end order is too long for k_deep_sortfam: re-run sorted
    EB_SCANWAIT = 1u << 16,   // a single-pass scan's look-back waited past its bound (k_scan_one)
};

// ---- device bounds checks (debug build: -DCC_DEBUG_BOUNDS, libccamd_debug.so) -----------------
// A checked index outside [0, n) records its site and value in g_dbg_fault (the first one wins) and is
// replaced by 0, so the kernel goes on reading valid memory; cc_debug_check reports it.  The release
// build compiles the checks away.
#ifdef CC_DEBUG_BOUNDS
__device__ unsigned long long g_dbg_fault;
__device__ __noinline__ int64_t dbg_fail(int site, int64_t i) {
    atomicCAS(&g_dbg_fault, 0ULL, ((unsigned long long)site << 48) | ((unsigned long long)i & 0xffffffffffffULL));
    return 0;
}
__device__ __forceinline__ int64_t dbg_idx(int64_t i, int64_t n, int site) {
    return (i < 0 || i >= n) ? dbg_fail(site, i) : i;
}
#define CC_IDX(i, n, site) ((std::remove_cv_t<std::remove_reference_t<decltype(i)>>)dbg_idx((int64_t)(i), (int64_t)(n), (site)))
#else
#define CC_IDX(i, n, site) (i)
#endif
enum : int {   // bounds-check sites (cc_debug_check's message)
    DS_REC = 1, DS_QNAME = 2, DS_PAYLOAD = 3, DS_SLOT = 4, DS_PAIR = 5, DS_MEMBER = 6, DS_VOTE_REC = 7,
};

struct TagKey {  // unique_tag fields (consensus_helper.py:295-304); bits = orient | readnum<<1 | run<<3
    int32_t bc, tid, pos, mtid, mpos, cigA, cigB;
    uint32_t bits;
};
struct CKey {  // sscs_qname fields (consensus_helper.py:240-247)
    int32_t bc, tidLo, posLo, tidHi, posHi, cigA, cigB;
    uint32_t strand;   // 0 pos, 1 neg, 2 None ; | run << 2 when scoped
    uint32_t abstlen;
    uint32_t pad[3];
};

// A record's key fields in one 32-B line (built at upload, k_core_pack): the pair hashes read a
// pair's far end (a random record) in one load instead of eight column gathers
struct alignas(32) RecCore {
    int32_t tid, pos, mtid, mpos, tlen, cig, bc, flag;
};

struct DevTable {
    int64_t n;
    int32_t *tid, *pos, *mtid, *mpos, *tlen, *cig, *qlen, *lseq, *bc, *rg;
    uint16_t* flag;
    uint8_t *mapq, *rflags;
    uint64_t* qn_off;
    uint16_t* qn_len;
    uint64_t* qn_ol;     // per record qn_off << 16 | qn_len (one load where both are needed; k_qn_pack)
    RecCore* core;       // per record its key fields (k_core_pack)
    uint8_t* qn_blob;
    uint64_t* pay_off;
    uint8_t* payload;
    uint64_t pay_bytes, qn_bytes;   // blob sizes (the debug build's bounds checks)
    uint64_t* rdig;      // per record a digest of all its bytes (record equality, k_fam_dedup)
    uint4* meta;         // per record the vote's 16-B member record without the valid bit (pack_meta)
    uint64_t* rkey;      // per record its position key (pos_key; position groups, mate search)
    uint32_t* ebits;     // error bits of the table's columns (EB_TOO_LONG), ORed into every pass's word
    int32_t max_len;
    // position-bucket geometry of a coordinate-sorted table (rebuilt by every read_bam pass over it;
    // the SC join's family buckets, k_fam_bucket): bucket of (t, pos) = tbase[t] + (pos >> geom[0])
    int64_t* tbase;      // per tid, first bucket; tbase[ntid] = mapped buckets (the unmapped tail's bucket)
    int32_t* ext;        // per tid, the largest position (k_table_cols, sorted tables)
    int32_t* geom;       // device: [0] bucket width shift (k_bucket_geom)
    int32_t ntid;        // 1 + the largest tid of the table (host scan at upload: a size, not data work)
    int64_t bkt_cap;     // an upper bound of the bucket count (see k_bucket_geom)
};

// ---- per-pass table preparation -------------------------------------------------------------
// A nibble word (8 BAM base codes) holds a base outside A,C,G,T,N (codes 1, 2, 4, 8, 15: popcount
// 1 or 4) at an in-range position (bit 3 of each in-range nibble set in m88).
__device__ __forceinline__ uint32_t nib_irregular(uint32_t x, uint32_t m88) {
    uint32_t p = x - ((x >> 1) & 0x55555555u);
    p = (p & 0x33333333u) + ((p >> 2) & 0x33333333u);          // popcount per nibble, 0..4
    const uint32_t a = p ^ 0x11111111u, b = p ^ 0x44444444u;    // 0 where popcount is 1 / 4 (all < 8)
    const uint32_t za = ~((a | 0x88888888u) - 0x11111111u) & 0x88888888u;
    const uint32_t zb = ~((b | 0x88888888u) - 0x11111111u) & 0x88888888u;
    return ~(za | zb) & m88;
}
// bit 3 of the nibbles of word w (bases 8w .. 8w+7 of a 32-base chunk) below nbase
__device__ __forceinline__ uint32_t nib_mask(int nbase, int w) {
    int vb = nbase - 8 * w;
    vb = vb < 0 ? 0 : (vb > 8 ? 8 : vb);
    const int full = vb >> 1;                                    // bytes with both nibbles in range
    uint32_t m = full >= 4 ? 0x88888888u : (((1u << (8 * full)) - 1u) & 0x88888888u);
    if ((vb & 1) && full < 4) m |= 0x80u << (8 * full);          // the high nibble comes first
    return m;
}

// Per record the votes' 16-B member record (pack_meta), from the SoA columns, one record per thread
// (coalesced): x = payload offset / 16, y = tlen, z = lseq | qlen << 16 (0xffff: no cigar),
// w = flag (12b) | mapq << 12 | rflags(3b) << 20 | rg7 << 24 (rg7 0x7f: no RG, 0x7e: id >= 126).
// On a sorted table also each tid's largest position (the bucket geometry's input).
constexpr int BC_T = 256;
__device__ __forceinline__ uint64_t pos_key(int32_t tid, int32_t pos) {
    return ((uint64_t)(uint32_t)(tid < 0 ? -1 : tid) << 32) | (uint64_t)(uint32_t)pos;
}

// A sorted table's position groups of more than DEEP_MIN - 1 records ("deep": more than the local
// kernels' 64): their first records are listed (any order) for the mate search's per-group qname
// buckets (k_deep_qsort).
constexpr int DEEP_MIN = 65;
// The table's derived columns, once per upload (they depend on the records only): each record's
// 16-B member record, its position key, its tid's largest position (sorted tables: the last record of
// a tid run; unused otherwise), and the column-width error bit.
__global__ __launch_bounds__(BC_T) void k_table_cols(DevTable T) {
    const int64_t r = (int64_t)blockIdx.x * BC_T + threadIdx.x;
    if (r >= T.n) return;
    const uint64_t po = T.pay_off[r];
    const int32_t ls = T.lseq[r], ql = T.qlen[r];
#ifdef CC_DEBUG_BOUNDS
    // the record's payload slot [qual, pad16][nibbles, pad16] lies inside the blob
    if (po + (uint64_t)((ls + 15) & ~15) + (uint64_t)(((ls + 1) / 2 + 15) & ~15) > T.pay_bytes + 64) dbg_fail(DS_PAYLOAD, r);
#endif
    if (ls > 0xffff || ql > 0xfffe || (po >> 4) > 0xffffffffULL) atomicOr(T.ebits, EB_TOO_LONG);
    const uint32_t lq = (uint32_t)(ls & 0xffff) | ((uint32_t)(ql < 0 ? 0xffff : ql) << 16);
    const int32_t rg = T.rg[r];
    const uint32_t rg7 = rg < 0 ? 0x7fu : (rg >= 126 ? 0x7eu : (uint32_t)rg);
    const uint32_t w = ((uint32_t)T.flag[r] & 0xfffu) | ((uint32_t)T.mapq[r] << 12) | ((uint32_t)(T.rflags[r] & 7u) << 20) |
                       (rg7 << 24);
    T.meta[r] = make_uint4((uint32_t)(po >> 4), (uint32_t)T.tlen[r], lq, w);
    const int32_t t = T.tid[r], p = T.pos[r];
    if (t >= 0 && t < T.ntid && (r + 1 == T.n || T.tid[r + 1] != t)) T.ext[t] = p < 0 ? 0 : p;
    T.rkey[r] = pos_key(t, p);
}

// The per-pass part of the table preparation: the deep position groups' list (sorted tables), the
// record -> read end map's reset, and the table's column error bits into the pass's word.
__device__ __forceinline__ void build_meta_rec(const DevTable& T, int32_t* __restrict__ rec_e, uint32_t* __restrict__ err,
                                               int32_t* __restrict__ dlist, uint32_t* __restrict__ ndeep, int64_t dcap) {
    const int64_t r = (int64_t)blockIdx.x * BC_T + threadIdx.x;
    if (r == 0) {
        const uint32_t eb = *T.ebits;
        if (eb) atomicOr(err, eb);
    }
    if (dlist) {   // every lane reaches the wave's append
        bool dp = false;
        if (r < T.n) {
            const int32_t t = T.tid[r], p = T.pos[r];
            const bool start = r == 0 || T.tid[r - 1] != t || T.pos[r - 1] != p;
            const int64_t q = r + DEEP_MIN - 1;
            dp = start && q < T.n && T.tid[q] == t && T.pos[q] == p;
        }
        const uint64_t m = __ballot(dp);
        if (m) {
            const int lane = threadIdx.x & 63;
            uint32_t base = 0;
            if (lane == __ffsll((unsigned long long)m) - 1) base = atomicAdd(ndeep, (uint32_t)__popcll(m));
            base = __shfl(base, __ffsll((unsigned long long)m) - 1, 64);
            if (dp) {
                const uint32_t o = base + (uint32_t)__popcll(m & ((1ULL << lane) - 1ULL));
                if ((int64_t)o < dcap) dlist[o] = (int32_t)r;
                else atomicOr(err, EB_PLAN);
            }
        }
    }
    if (r < T.n && rec_e) rec_e[r] = -1;   // (set by the pair scan on sorted tables)
}
__global__ __launch_bounds__(BC_T) void k_build_meta(DevTable T, int32_t* __restrict__ rec_e, uint32_t* __restrict__ err,
                                                     int32_t* __restrict__ dlist, uint32_t* __restrict__ ndeep,
                                                     int64_t dcap) {
    build_meta_rec(T, rec_e, err, dlist, ndeep, dcap);
}

// Bucket geometry of a coordinate-sorted table from each tid's largest position (one block): the
// finest power-of-two width with at most about two buckets per record (sum_t (ext[t] >> s) + 1 <=
// 2N + ntid, else s = 30, where the count is <= 2 ntid), and the per-tid first buckets.
constexpr int BG_T = 1024;
__device__ __forceinline__ int64_t block_sum64(int64_t v, int64_t* s_w) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();
    if (lane == 0) s_w[w] = v;
    __syncthreads();
    int64_t tot = 0;
#pragma unroll
    for (int j = 0; j < BG_T / 64; ++j) tot += s_w[j];
    return tot;
}
__global__ __launch_bounds__(BG_T) void k_bucket_geom(int64_t N, int32_t ntid, const int32_t* __restrict__ ext,
                                                      int64_t* __restrict__ tbase, int32_t* __restrict__ geom) {
    __shared__ int64_t s_w[BG_T / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int bs = 30;
    for (int s = 0; s < 30; ++s) {
        int64_t part = 0;
        for (int32_t x = t; x < ntid; x += BG_T) part += ((int64_t)ext[x] >> s) + 1;
        if (block_sum64(part, s_w) <= 2 * N + ntid) { bs = s; break; }
    }
    int64_t carry = 0;
    for (int32_t base = 0; base < ntid; base += BG_T) {
        const int32_t x = base + t;
        int64_t inc = x < ntid ? ((int64_t)ext[x] >> bs) + 1 : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        __syncthreads();
        if (lane == 63) s_w[w] = inc;
        __syncthreads();
        int64_t pre = 0, all = 0;
#pragma unroll
        for (int j = 0; j < BG_T / 64; ++j) {
            if (j < w) pre += s_w[j];
            all += s_w[j];
        }
        if (x < ntid) tbase[x + 1] = carry + pre + inc;
        carry += all;
    }
    if (t == 0) { tbase[0] = 0; geom[0] = bs; geom[1] = 0; }
}

// ------------------------------------------------------------------ hashing
__device__ __forceinline__ uint64_t mix64(uint64_t h) {
    h ^= h >> 31;
    h *= 0x7fb5d329728ea185ULL;
    h ^= h >> 27;
    h *= 0x81dadef4bc2dd44dULL;
    h ^= h >> 33;
    return h;
}
__device__ __forceinline__ uint64_t hcomb(uint64_t h, uint64_t w) {
    return mix64(h ^ (w + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2)));
}
__device__ __forceinline__ uint64_t clamp_key(uint64_t h) { return h == ~0ULL ? ~0ULL - 1 : h; }

__device__ __forceinline__ uint64_t hash_tag(const TagKey& k, uint64_t seed) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(&k);
    uint64_t h = seed;
#pragma unroll
    for (int i = 0; i < 4; ++i) h = hcomb(h, w[i]);
    return clamp_key(h);
}
__device__ __forceinline__ uint64_t hash_ckey(const CKey& k, uint64_t seed) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(&k);
    uint64_t h = seed ^ 0x51ed270b27d4a3c5ULL;
#pragma unroll
    for (int i = 0; i < 5; ++i) h = hcomb(h, w[i]);
    return clamp_key(h);
}
__device__ __forceinline__ bool tag_eq(const TagKey& a, const TagKey& b) {
    return a.bc == b.bc && a.tid == b.tid && a.pos == b.pos && a.mtid == b.mtid && a.mpos == b.mpos &&
           a.cigA == b.cigA && a.cigB == b.cigB && a.bits == b.bits;
}
__device__ __forceinline__ bool ckey_eq(const CKey& a, const CKey& b) {
    return a.bc == b.bc && a.tidLo == b.tidLo && a.posLo == b.posLo && a.tidHi == b.tidHi && a.posHi == b.posHi &&
           a.cigA == b.cigA && a.cigB == b.cigB && a.strand == b.strand && a.abstlen == b.abstlen;
}

// which_read (consensus_helper.py:57-81): 0 R1, 1 R2, 2 None
__device__ __forceinline__ int which_read(int f) {
    switch (f) {
        case 99: case 83: case 67: case 115: case 81: case 97: case 65: case 113: return 0;
        case 147: case 163: case 131: case 179: case 161: case 145: case 129: case 177: return 1;
        default: return 2;
    }
}
// which_strand (consensus_helper.py:84-156): 0 pos, 1 neg, 2 None
__device__ __forceinline__ int which_strand(int f, int tid, int mtid, int pos, int mpos) {
    switch (f) {
        case 99: case 147: case 67: case 131: return 0;
        case 83: case 163: case 115: case 179: return 1;
        case 65: case 129: case 113: case 177: case 81: case 161: case 97: case 145: {
            int rn = which_read(f);
            bool p = (tid < mtid && rn == 0) || (tid > mtid && rn == 1) || (tid == mtid && rn == 0 && pos < mpos) ||
                     (tid == mtid && rn == 1 && pos > mpos);
            return p ? 0 : 1;
        }
        default: return 2;
    }
}
__device__ __forceinline__ bool mate_unmapped_flag(int f) {
    return f == 73 || f == 89 || f == 121 || f == 153 || f == 185 || f == 137;
}

// The completed pairs of a read_bam pass (written in the pair scan's store phase, EmitPairs): the
// records of the first and second end, and the region that completed the pair.  Tags and consensus
// keys are recomputed from the records where they are compared or emitted instead of being
// materialised per read end (k_pair_keys writes only their hashes).
struct PairView {
    const int32_t *rec1, *rec2, *region;
    const int32_t* region_run;
    int scoped;
    const int4* tag;   // per pair the tag fields both ends share {bc, cigA, cigB, run} (k_pair_keys)
};
__device__ __forceinline__ uint32_t pair_run(const PairView& V, int32_t p) {
    return V.scoped ? (uint32_t)V.region_run[V.region[p]] : 0u;
}

// unique_tag (consensus_helper.py:295-304) of end i of the pair (a, b): barcode of the first read,
// the end's own coordinates, the pair's cigars in cigar_order (consensus_helper.py:159-196), and
// orientation | which_read << 1 | run << 3
__device__ __forceinline__ TagKey make_tag(const DevTable& T, int32_t a, int32_t b, int i, uint32_t run) {
    a = CC_IDX(a, T.n, DS_REC);
    b = CC_IDX(b, T.n, DS_REC);
    const int fa = T.flag[a];
    const int rnA = which_read(fa);
    const int stA = which_strand(fa, T.tid[a], T.mtid[a], T.pos[a], T.mpos[a]);
    const int ca = T.cig[a], cb = T.cig[b];
    const bool keep = (stA == 0 && rnA == 0) || (stA == 1 && rnA == 1);
    const int32_t r = i ? b : a;
    const int f = i ? (int)T.flag[b] : fa;
    TagKey t;
    t.bc = T.bc[a];
    t.tid = T.tid[r]; t.pos = T.pos[r]; t.mtid = T.mtid[r]; t.mpos = T.mpos[r];
    t.cigA = keep ? ca : cb;
    t.cigB = keep ? cb : ca;
    t.bits = (uint32_t)((f >> 4) & 1) | ((uint32_t)which_read(f) << 1) | (run << 3);
    return t;
}
// the same tag from the end's own record r and its pair's shared fields (make_tag's values)
__device__ __forceinline__ TagKey tag_of_rec(const DevTable& T, int32_t r, int4 pt) {
    r = CC_IDX(r, T.n, DS_REC);
    const int f = T.flag[r];
    TagKey t;
    t.bc = pt.x;
    t.tid = T.tid[r]; t.pos = T.pos[r]; t.mtid = T.mtid[r]; t.mpos = T.mpos[r];
    t.cigA = pt.y;
    t.cigB = pt.z;
    t.bits = (uint32_t)((f >> 4) & 1) | ((uint32_t)which_read(f) << 1) | ((uint32_t)pt.w << 3);
    return t;
}
// the same without the record's (tid, pos) (zero): for two records known to share them
__device__ __forceinline__ TagKey tag_of_rec_np(const DevTable& T, int32_t r, int4 pt) {
    r = CC_IDX(r, T.n, DS_REC);
    const int f = T.flag[r];
    TagKey t;
    t.bc = pt.x;
    t.tid = 0; t.pos = 0; t.mtid = T.mtid[r]; t.mpos = T.mpos[r];
    t.cigA = pt.y;
    t.cigB = pt.z;
    t.bits = (uint32_t)((f >> 4) & 1) | ((uint32_t)which_read(f) << 1) | ((uint32_t)pt.w << 3);
    return t;
}
__device__ __forceinline__ TagKey tag_of_end(const DevTable& T, const PairView& V, uint32_t e) {
    const int32_t p = (int32_t)(e >> 1);
    return tag_of_rec(T, (e & 1u) ? V.rec2[p] : V.rec1[p], V.tag[p]);
}

// sscs_qname's consensus key (consensus_helper.py:240-247) of the pair (a, b); pads zero (hashed)
__device__ __forceinline__ CKey make_ckey(const DevTable& T, int32_t a, int32_t b, uint32_t run) {
    a = CC_IDX(a, T.n, DS_REC);
    b = CC_IDX(b, T.n, DS_REC);
    const int fa = T.flag[a];
    const int ta = T.tid[a], tb = T.tid[b], pa = T.pos[a], pb = T.pos[b];
    const int rnA = which_read(fa);
    const int stA = which_strand(fa, ta, T.mtid[a], pa, T.mpos[a]);
    const int ca = T.cig[a], cb = T.cig[b];
    const bool keep = (stA == 0 && rnA == 0) || (stA == 1 && rnA == 1);
    CKey c;
    int rc = ta, mc = tb, rp = pa, mp = pb;
    if ((rc == mc && rp > mp) || rc > mc) { rc = tb; mc = ta; rp = pb; mp = pa; }
    c.bc = T.bc[a]; c.tidLo = rc; c.posLo = rp; c.tidHi = mc; c.posHi = mp;
    c.cigA = keep ? ca : cb;
    c.cigB = keep ? cb : ca;
    c.strand = (uint32_t)stA | (run << 2);
    const int tl = T.tlen[a];
    c.abstlen = tl < 0 ? (uint32_t)(-(int64_t)tl) : (uint32_t)tl;
    c.pad[0] = c.pad[1] = c.pad[2] = 0;
    return c;
}
// make_tag / make_ckey from the two records' cores (the same values)
__device__ __forceinline__ TagKey make_tag_c(const RecCore& A, const RecCore& B, int i, uint32_t run) {
    const int rnA = which_read(A.flag);
    const int stA = which_strand(A.flag, A.tid, A.mtid, A.pos, A.mpos);
    const bool keep = (stA == 0 && rnA == 0) || (stA == 1 && rnA == 1);
    const RecCore& R = i ? B : A;
    TagKey t;
    t.bc = A.bc;
    t.tid = R.tid; t.pos = R.pos; t.mtid = R.mtid; t.mpos = R.mpos;
    t.cigA = keep ? A.cig : B.cig;
    t.cigB = keep ? B.cig : A.cig;
    t.bits = (uint32_t)((R.flag >> 4) & 1) | ((uint32_t)which_read(R.flag) << 1) | (run << 3);
    return t;
}
__device__ __forceinline__ CKey make_ckey_c(const RecCore& A, const RecCore& B, uint32_t run) {
    const int rnA = which_read(A.flag);
    const int stA = which_strand(A.flag, A.tid, A.mtid, A.pos, A.mpos);
    const bool keep = (stA == 0 && rnA == 0) || (stA == 1 && rnA == 1);
    CKey c;
    int rc = A.tid, mc = B.tid, rp = A.pos, mp = B.pos;
    if ((rc == mc && rp > mp) || rc > mc) { rc = B.tid; mc = A.tid; rp = B.pos; mp = A.pos; }
    c.bc = A.bc; c.tidLo = rc; c.posLo = rp; c.tidHi = mc; c.posHi = mp;
    c.cigA = keep ? A.cig : B.cig;
    c.cigB = keep ? B.cig : A.cig;
    c.strand = (uint32_t)stA | (run << 2);
    c.abstlen = A.tlen < 0 ? (uint32_t)(-(int64_t)A.tlen) : (uint32_t)A.tlen;
    c.pad[0] = c.pad[1] = c.pad[2] = 0;
    return c;
}
__global__ __launch_bounds__(256) void k_core_pack(int64_t n, DevTable T) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    RecCore c;
    c.tid = T.tid[r]; c.pos = T.pos[r]; c.mtid = T.mtid[r]; c.mpos = T.mpos[r];
    c.tlen = T.tlen[r]; c.cig = T.cig[r]; c.bc = T.bc[r]; c.flag = T.flag[r];
    T.core[r] = c;
}

__device__ __forceinline__ CKey ckey_of_pair(const DevTable& T, const PairView& V, int32_t p) {
    return make_ckey_c(T.core[CC_IDX(V.rec1[p], T.n, DS_REC)], T.core[CC_IDX(V.rec2[p], T.n, DS_REC)], pair_run(V, p));
}

__device__ __forceinline__ uint64_t qname_hash(const DevTable& T, int32_t r, uint64_t seed) {
    r = CC_IDX(r, T.n, DS_REC);
    const uint64_t* w = reinterpret_cast<const uint64_t*>(T.qn_blob + CC_IDX(T.qn_off[r], T.qn_bytes + 1, DS_QNAME));
    const int len = T.qn_len[r];
    const int nw = (len + 7) / 8;
    // the words of typical qnames loaded together, then chained in order
    uint64_t v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = i < nw ? w[i] : 0ULL;
    uint64_t h = seed;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < nw) h = hcomb(h, v[i]);
    for (int i = 4; i < nw; ++i) h = hcomb(h, w[i]);
    return hcomb(h, (uint64_t)len);
}
__global__ __launch_bounds__(256) void k_qn_pack(int64_t n, const uint64_t* __restrict__ off,
                                                 const uint16_t* __restrict__ len, uint64_t* __restrict__ ol) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) ol[r] = (off[r] << 16) | len[r];
}
__device__ __forceinline__ bool qname_eq(const DevTable& T, int32_t a, int32_t b) {
    // lengths and offsets loaded together (one packed word per record); the words of the shorter
    // slot compared (a length mismatch is a difference by itself)
    a = CC_IDX(a, T.n, DS_REC);
    b = CC_IDX(b, T.n, DS_REC);
    const uint64_t oa = T.qn_ol[a], ob = T.qn_ol[b];
    const int la = (int)(oa & 0xffffu), lb = (int)(ob & 0xffffu);
    const uint64_t* wa = reinterpret_cast<const uint64_t*>(T.qn_blob + CC_IDX(oa >> 16, T.qn_bytes + 1, DS_QNAME));
    const uint64_t* wb = reinterpret_cast<const uint64_t*>(T.qn_blob + CC_IDX(ob >> 16, T.qn_bytes + 1, DS_QNAME));
    const int nw = ((la < lb ? la : lb) + 7) >> 3;
    uint64_t d = la != lb ? 1ULL : 0ULL;
#pragma unroll
    for (int i = 0; i < 4; ++i)   // the words of typical qnames loaded together
        if (i < nw) d |= wa[i] ^ wb[i];
    for (int i = 4; i < nw && !d; ++i) d |= wa[i] ^ wb[i];
    return d == 0;
}

__device__ __forceinline__ int32_t readlane_i32(int32_t v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int k) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, k);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), k);
    return ((uint64_t)hi << 32) | lo;
}

// Block index remapped so that each XCD walks one contiguous run of blocks: workgroups are dealt
// round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch), so blocks b and b + 8
// share an L2.  Kernels whose threads re-read records a few hundred entries back (mates, position
// groups) then find them in their own XCD's L2.  A bijection on [0, gridDim.x); speed only.
__device__ __forceinline__ int64_t xcd_block() {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t q = nb >> 3, rem = nb & 7u, x = b & 7u;
    return (int64_t)(x * q + (x < rem ? x : rem) + (b >> 3));
}

constexpr int GRP_SMALL = 64;   // position groups up to this size are handled locally

// Add a per-lane count to a device total: wave sum, one atomic per wave.  Every lane of the wave
// must reach it (no early return before it).
__device__ __forceinline__ void wave_add(uint32_t v, uint32_t* dst) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, v);
}

// A count most waves contribute to (c4: nearly every read is residual / in a deep group): one
// atomic per wave on one address serialises on its L2 line, so the waves add into 64 stripes 64 B
// apart and k_stripe_total folds them into the plan slot (and zeroes them for the next pass).
constexpr int PSTRIPES = 64, PSTRIDE = 16;
__device__ __forceinline__ void stripe_add(uint32_t v, uint32_t* stripes) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(stripes + PSTRIDE * (w & (PSTRIPES - 1)), v);
}

__global__ __launch_bounds__(64) void k_stripe_total(uint32_t* __restrict__ stripes, uint32_t* __restrict__ total) {
    const int t = threadIdx.x;
    uint32_t v = stripes[PSTRIDE * t];
    stripes[PSTRIDE * t] = 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (t == 0) *total = v;
}

// Several fills of 32-bit words in one launch (the per-pass zeroing of counters, error words and
// tables): a memset is a dispatch of its own, ~4 us each even for 4 bytes.
struct FillSet {
    static constexpr int K = 8;
    uint32_t* p[K];
    int64_t n[K];    // words
    uint32_t v[K];
    int k;
};
__global__ __launch_bounds__(256) void k_fill(FillSet fs) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int d = 0; d < fs.k; ++d) {
        uint32_t* p = fs.p[d];
        const int64_t n = fs.n[d];
        const int64_t n4 = ((uintptr_t)p & 15u) ? 0 : n >> 2;   // 16-B stores where the start allows
        const uint32_t v = fs.v[d];
        uint4* p4 = reinterpret_cast<uint4*>(p);
        for (int64_t i = t; i < n4; i += stride) p4[i] = make_uint4(v, v, v, v);
        for (int64_t i = 4 * n4 + t; i < n; i += stride) p[i] = v;
    }
}

// ------------------------------------------------------------------ read_bam kernels
// The counters are striped over CNT_STRIPES copies (by block index) so that a launch of many
// blocks does not serialise on one address; the end-of-pass readback sums the stripes.
constexpr int CNT_STRIPES = 64;
__device__ __forceinline__ unsigned long long* cnt_stripe(unsigned long long* cnt) {
    return cnt + CC_NUM_COUNTERS * (blockIdx.x & (CNT_STRIPES - 1));
}

// Sum per-thread counters over the workgroup (wave shuffles + LDS) and add them to the block's
// counter stripe with one atomic per workgroup and counter.
template <int NC>
__device__ __forceinline__ void block_count(int (&v)[NC], const int (&slot)[NC], unsigned long long* cnt) {
    __shared__ int s_red[4][NC];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        int x = v[c];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o);
        if (lane == 0) s_red[wv][c] = x;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NC; ++c)   // compile-time indices: the arrays stay in registers
        if ((int)threadIdx.x == c) {
            int t = 0;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += s_red[w][c];
            if (t) atomicAdd(&cnt_stripe(cnt)[slot[c]], (unsigned long long)t);
        }
}


// The filters of consensus_helper.py:404-420 and the qname key of stream entry s (record r, region
// word reg_w): the pairing arrays' initial values and the counters (acc: unmapped, mate-unmapped,
// secondary/supplementary, bad spacer, bad-listed, uncounted).
struct ClassifyOut {
    uint64_t* skey;
    uint32_t* sval;      // the qname sort's values (not needed by the coordinate search)
    uint8_t* badflag;    // only a pass that lists bad reads keeps the flags
    int32_t *mate_of, *partner, *claimer;
    uint8_t* pflag;
};
__device__ __forceinline__ void classify_entry(int64_t s, int32_t r, int32_t reg, const int32_t* __restrict__ region_run,
                                               const DevTable& T, int delim_filter, int badread, int scoped,
                                               uint64_t seed, const ClassifyOut& o, int (&acc)[6]) {
    // multi-GPU shards: a first-streamed end whose pair completes on another shard is moved there
    // (a foreign entry, region -(r+1), on the receiver; the moved bit on the sender's own entry)
    const bool foreign = reg < 0;
    const bool moved = !foreign && (reg & CC_REGION_MOVED);
    if (foreign) reg = -reg - 1;
    else reg &= ~CC_REGION_MOVED;
    const int f = T.flag[r];
    const uint8_t rf = T.rflags[r];
    int c;
    if (delim_filter && (rf & CC_RF_BAD_SPACER)) c = 1;
    else if (f & 4) c = 2;
    else if (mate_unmapped_flag(f)) c = 3;
    else if (f & 0x100) c = 4;
    else if (f & 0x800) c = 4;
    else c = 0;
    // The record pairs (pair_dict) unless it is a bad read of a pass that lists them; a listed
    // bad read is listed and counted by its owner.  Every other record is counted (and paired)
    // where its pair completes: the receiver for a moved one.
    const bool inpair0 = (c == 0) || !badread;
    const bool listed = !inpair0 && !foreign;
    const bool counted = foreign ? inpair0 : (moved ? !inpair0 : true);
    const bool inpair = inpair0 && !moved;
    if (o.badflag) o.badflag[s] = listed ? 1 : 0;
    // branch-free sums: an if-chain over acc[] is turned into one dynamically indexed add (scratch)
    const int cn = counted ? 1 : 0;
    acc[0] += cn & (c == 2);
    acc[1] += cn & (c == 3);
    acc[2] += cn & (c == 4);
    acc[3] += cn & (c == 1);
    acc[4] += cn & (listed ? 1 : 0);
    acc[5] += 1 - cn;
    uint64_t k = ~0ULL;
    if (inpair) {
        uint64_t h = qname_hash(T, r, seed);
        if (scoped) h = hcomb(h, (uint64_t)(uint32_t)region_run[reg] + 1);
        k = clamp_key(h);
    }
    o.skey[s] = k;
    if (o.sval) o.sval[s] = (uint32_t)s;
    o.mate_of[s] = -1;
    o.pflag[s] = 0;   // 1 where a pair completes (k_pair_coord_tile / k_pair_mark): the pair list's flags
    if (o.claimer) o.claimer[s] = -1;
    if (o.partner) o.partner[s] = -1;   // identity streams: the tiled mate search writes every entry's
}
__device__ __forceinline__ void classify_count(int (&acc)[6], unsigned long long* __restrict__ cnt) {
    const int slots[6] = {CC_CNT_UNMAPPED, CC_CNT_UNMAPPED_MATE, CC_CNT_MULTIPLE_MAPPING, CC_CNT_BAD_SPACER,
                          CC_CNT_BAD_LISTED, CC_CNT_FOREIGN};
    block_count<6>(acc, slots, cnt);
}

// ident: the stream is the table in file order (stream_rec[s] == s), the read_bam of a whole
// BAM without a bed file; the kernels then skip the stream_rec gather (one dependent load).
__global__ __launch_bounds__(256) void k_classify(int64_t S, int ident, const int32_t* __restrict__ stream_rec,
                                                  const int32_t* __restrict__ stream_region,
                                                  const int32_t* __restrict__ region_run, DevTable T, int delim_filter,
                                                  int badread, int scoped, uint64_t seed, ClassifyOut o,
                                                  unsigned long long* __restrict__ cnt) {
    int acc[6] = {0, 0, 0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < S; s += stride) {
        const int32_t r = ident ? (int32_t)s : stream_rec[s];
        classify_entry(s, r, stream_region[s], region_run, T, delim_filter, badread, scoped, seed, o, acc);
    }
    classify_count(acc, cnt);
}

// The per-pass table preparation of k_build_meta and k_classify in one pass over the records, for an
// identity stream (the records in file order: every bench pass without a bed file) on a sorted table:
// each record's member record, position key, read-end map, its tid's extent, the deep-group list,
// and as its own stream entry its filters, qname key and pairing arrays.
__global__ __launch_bounds__(BC_T) void k_build_meta_cls(DevTable T, int32_t* __restrict__ rec_e, uint32_t* __restrict__ err,
                                                         int32_t* __restrict__ dlist, uint32_t* __restrict__ ndeep,
                                                         int64_t dcap, const int32_t* __restrict__ stream_region,
                                                         const int32_t* __restrict__ region_run, int delim_filter,
                                                         int badread, int scoped, uint64_t seed, ClassifyOut o,
                                                         unsigned long long* __restrict__ cnt) {
    build_meta_rec(T, rec_e, err, dlist, ndeep, dcap);
    int acc[6] = {0, 0, 0, 0, 0, 0};
    const int64_t r = (int64_t)blockIdx.x * BC_T + threadIdx.x;
    if (r < T.n) classify_entry(r, (int32_t)r, stream_region[r], region_run, T, delim_filter, badread, scoped, seed, o, acc);
    classify_count(acc, cnt);
}

// pair_dict (consensus_helper.py:426-432) over qname keys sorted stably by (key, stream position):
// the occurrences of one qname pair up in stream order, (1st, 2nd), (3rd, 4th), ...; an odd last one
// stays in pair_dict.  A qname seen more than twice counts in n_multi (record equality then matters
// for the "line read twice" rule, k_fam_dedup).
__global__ __launch_bounds__(256) void k_pair_mark(int64_t S, const uint64_t* __restrict__ key,
                                                   const uint32_t* __restrict__ val, int ident,
                                                   const int32_t* __restrict__ stream_rec, DevTable T,
                                                   int32_t* __restrict__ mate_of, uint8_t* __restrict__ pflag,
                                                   uint32_t* __restrict__ err,
                                                   unsigned long long* __restrict__ cnt, uint32_t* __restrict__ n_multi) {
    // one sorted entry per thread (c4: ~50 M residual entries; a grid-stride loop would serialise
    // each thread's dependent qname loads), the counts through stripes and per-block atomics
    int acc[1] = {0};
    uint32_t multi = 0;
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < S) {
        const uint64_t k = key[j];
        if (k != ~0ULL && (j == 0 || key[j - 1] != k)) {
            int64_t m = 1;
            while (j + m < S && key[j + m] == k) ++m;
            if (m == 1) {
                acc[0] += 1;
            } else {
                // identity streams: the stream slot is the record (no stream_rec gather in the chain)
                const int32_t r0 = ident ? (int32_t)val[j] : stream_rec[val[j]];
                bool same = true;
                for (int64_t i = 1; i < m && same; ++i)
                    same = qname_eq(T, r0, ident ? (int32_t)val[j + i] : stream_rec[val[j + i]]);
                if (!same) {
                    atomicOr(err, EB_COLLISION);
                } else {
                    for (int64_t i = 0; i + 1 < m; i += 2) {
                        mate_of[val[j + i + 1]] = (int32_t)val[j + i];
                        pflag[val[j + i + 1]] = 1;
                    }
                    acc[0] += (int)(m & 1);
                    multi = m > 2 ? 1u : 0u;
                }
            }
        }
    }
    stripe_add(multi, n_multi);
    const int slots[1] = {CC_CNT_UNPAIRED};
    block_count<1>(acc, slots, cnt);
}

// ---- position buckets (coordinate-sorted tables; the SC join's family buckets) ------------
__device__ __forceinline__ int64_t bucket_of(const int64_t* __restrict__ tbase, int32_t ntid, int32_t bshift,
                                             int32_t t, int32_t p) {
    if (t < 0 || t >= ntid) return tbase[ntid];
    const int64_t b = tbase[t] + ((p < 0 ? 0 : p) >> bshift);
    return b < tbase[t + 1] ? b : tbase[t + 1];
}

// ---- pairing by mate coordinates (coordinate-sorted tables) -------------------------------
// pair_dict pairs mates by qname (consensus_helper.py:426-432).  In a sorted table the mate of a
// read lies in the position group (mtid, mpos): gallop there from the read's own index and look
// for the one in-pairing record with the same qname key; the qname bytes are then compared.
// Reads whose mate is not found that way go to the exact sort path (the residual).
__global__ __launch_bounds__(256) void k_scatter_stream(int64_t S, int ident, const int32_t* __restrict__ stream_rec,
                                                        const uint64_t* __restrict__ skey,
                                                        int32_t* __restrict__ spos, uint64_t* __restrict__ rq) {
    int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const int32_t r = ident ? (int32_t)s : stream_rec[s];
    spos[r] = (int32_t)s;
    rq[r] = skey[s];
}

constexpr int32_t PD_W = 512;        // pairs spanning more stream entries go to the global table
constexpr int64_t PD_TILE = 2048;     // stream entries per k_pair_resid block (plus PD_W before)
constexpr int PD_SLOTS = 4096;        // LDS table: at most PD_TILE + PD_W found-pair ends enter
// a table entry: 20 fingerprint bits of the key over the later end's offset from the block's window
// start (< PD_TILE + 2 PD_W, 12 bits): 16 KB of LDS, full occupancy
static_assert(PD_TILE + 2 * PD_W <= 4095, "k_pair_resid's entry offsets take 12 bits");

// ---- deep position groups: each group's records bucketed by qname key ----------------------
// The mate search walks a target position group of at most GRP_SMALL + 1 records; in deeper groups
// (targeted panels, config C4: thousands of reads per position) it looks the key up instead: one
// block per deep group buckets the group's records by the top bits of their qname key in one
// counting pass (histogram, scan and scatter in LDS) into gq over the group's own index range
// [g0, g1), with the bucket offsets in boff over the same range; gend[g0] = g1 (-1 - g1 when the
// group has more than DQ_CAP records: those stay on the exact sort path), and the group's position
// key enters a small table (dg_insert) that the search finds it by.  A segmented pass over ranges
// the table already has: no scatter across groups, no global sort.
constexpr int DQ_CAP = 16384, DQ_T = 1024;

// the end of the position group starting at g0 (rkey[g0] = its key): 1024 probes 16 apart, then 16
__device__ __forceinline__ int64_t deep_group_end(int64_t N, const uint64_t* __restrict__ rkey, int64_t g0,
                                                  int64_t* s_min) {
    const uint64_t k = rkey[g0];
    const int t = threadIdx.x;
    if (t == 0) *s_min = INT64_MAX;
    __syncthreads();
    {
        const int64_t x = g0 + 16 * (int64_t)(t + 1);
        if (x >= N || rkey[x] != k) atomicMin((unsigned long long*)s_min, (unsigned long long)(t + 1));
    }
    __syncthreads();
    const int64_t c = *s_min;   // first probe past the group (INT64_MAX: more than 16 * 1024 records)
    __syncthreads();
    if (c == INT64_MAX) {
        // a group beyond DQ_CAP: its end by a serial gallop (rare)
        if (t == 0) {
            int64_t lo = g0 + 16 * DQ_T, step = 16 * DQ_T, hi;
            for (;;) {
                hi = lo + step;
                if (hi >= N || rkey[hi] != k) break;
                lo = hi;
                step <<= 1;
            }
            if (hi > N) hi = N;
            while (lo + 1 < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (rkey[mid] == k) lo = mid;
                else hi = mid;
            }
            *s_min = hi;
        }
        __syncthreads();
        const int64_t e = *s_min;
        __syncthreads();
        return e;
    }
    if (t == 0) *s_min = INT64_MAX;
    __syncthreads();
    if (t < 16) {
        const int64_t x = g0 + 16 * (c - 1) + t + 1;   // the group's end lies in (16(c-1), 16c]
        if (x >= N || rkey[x] != k) atomicMin((unsigned long long*)s_min, (unsigned long long)x);
    }
    __syncthreads();
    const int64_t e = *s_min < N ? *s_min : N;
    __syncthreads();
    return e;
}

// The deep groups by position key (open addressing, DG_EMPTY free): the mate search finds a deep
// target group's first record here instead of searching the table for it.
constexpr uint64_t DG_EMPTY = 0xFFFFFFFEFFFFFFFEULL;   // tid -2, pos -2: no position key
// 16-B entries {position key, the group's first record | its gend entry (g1, or -1 - g1 when too
// deep to bucket) << 32}: one load gives the search the group's extent with its start
__device__ __forceinline__ void dg_insert(unsigned long long* __restrict__ hk, uint64_t mask, uint64_t key, int32_t g0,
                                          int32_t ge) {
    uint64_t h = mix64(key) & mask;
    for (uint64_t i = 0; i <= mask; ++i) {
        const unsigned long long prev = atomicCAS(&hk[2 * h], (unsigned long long)DG_EMPTY, (unsigned long long)key);
        if (prev == DG_EMPTY || prev == key) {
            hk[2 * h + 1] = (unsigned long long)(uint32_t)g0 | ((unsigned long long)(uint32_t)ge << 32);
            return;
        }
        h = (h + 1) & mask;
    }
}
__device__ __forceinline__ int2 dg_lookup(const unsigned long long* __restrict__ hk, uint64_t mask, uint64_t key) {
    uint64_t h = mix64(key) & mask;
    for (uint64_t i = 0; i <= mask; ++i) {
        const ulonglong2 e = reinterpret_cast<const ulonglong2*>(hk)[h];
        if (e.x == key) return make_int2((int32_t)(uint32_t)e.y, (int32_t)(uint32_t)(e.y >> 32));
        if (e.x == DG_EMPTY) return make_int2(-1, -1);
        h = (h + 1) & mask;
    }
    return make_int2(-1, -1);
}

__global__ __launch_bounds__(DQ_T) void k_deep_qsort(const uint32_t* __restrict__ ndeep, const int32_t* __restrict__ dlist,
                                                     int64_t N, const uint64_t* __restrict__ rkey,
                                                     const uint64_t* __restrict__ qkey, uint64_t* __restrict__ gq,
                                                     int32_t* __restrict__ gend, uint32_t* __restrict__ boff,
                                                     unsigned long long* __restrict__ dgk,
                                                     uint64_t dgmask, uint32_t* __restrict__ gid) {
    // a group's records bucketed by the top bits of their qname key (one counting pass: histogram,
    // scan, scatter; the key hashes are uniform): nb = pow2 >= n / 2 buckets, bucket b's entries at
    // gq[g0 + boff[g0 + b], g0 + boff[g0 + b + 1]) (any order inside a bucket: the search reads all
    // of it), entries (key >> 16) << 16 | offset in the group
    __shared__ uint32_t s_c[DQ_CAP / 2 + 1];
    __shared__ int64_t s_min;
    __shared__ uint32_t s_w[DQ_T / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t nd = *ndeep;
    for (uint32_t gi = blockIdx.x; gi < nd; gi += gridDim.x) {
        const int64_t g0 = dlist[gi];
        const int64_t g1 = deep_group_end(N, rkey, g0, &s_min);
        // every record's deep group (the deep ends' tag sort keys on it: families of one position
        // group come out side by side)
        for (int64_t r = g0 + t; r < g1; r += DQ_T) gid[r] = gi;
        const int n = (int)min<int64_t>(g1 - g0, (int64_t)DQ_CAP + 1);
        if (n > DQ_CAP) {
            if (t == 0) {
                gend[g0] = (int32_t)(-1 - g1);
                dg_insert(dgk, dgmask, rkey[g0], (int32_t)g0, (int32_t)(-1 - g1));
            }
            continue;
        }
        int lb = 5;
        while ((1 << lb) < (n + 1) / 2) ++lb;
        const int nb = 1 << lb;
        for (int b = t; b <= nb; b += DQ_T) s_c[b] = 0u;
        __syncthreads();
        for (int i = t; i < n; i += DQ_T) atomicAdd(&s_c[qkey[g0 + i] >> (64 - lb)], 1u);
        __syncthreads();
        // exclusive scan of the nb counts (each thread a contiguous run of them)
        const int per = (nb + DQ_T - 1) / DQ_T;
        const int b0 = t * per, b1 = min(nb, b0 + per);
        uint32_t run = 0;
        for (int b = b0; b < b1; ++b) run += s_c[b];
        uint32_t x = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_w[wv] = x;
        __syncthreads();
        uint32_t pre = x - run;
        for (int w = 0; w < wv; ++w) pre += s_w[w];
        for (int b = b0; b < b1; ++b) {
            const uint32_t c = s_c[b];
            s_c[b] = pre;
            boff[g0 + b] = pre;
            pre += c;
        }
        if (t == 0) boff[g0 + nb] = (uint32_t)n;
        __syncthreads();
        for (int i = t; i < n; i += DQ_T) {
            const uint64_t k = qkey[g0 + i];
            const uint32_t o = atomicAdd(&s_c[k >> (64 - lb)], 1u);
            gq[g0 + o] = ((k >> 16) << 16) | (uint64_t)i;
        }
        if (t == 0) {
            gend[g0] = (int32_t)g1;
            dg_insert(dgk, dgmask, rkey[g0], (int32_t)g0, (int32_t)g1);
        }
        __syncthreads();
    }
}

// The one record of the deep group starting at g0 with qname key `key` other than record r, from
// the key's bucket (k_deep_qsort); -1 when there is none or several, or the group was too deep to
// bucket (the exact sort path pairs those)
__device__ __forceinline__ int32_t deep_find(const uint64_t* __restrict__ gq, const int32_t* __restrict__ gend,
                                             const uint32_t* __restrict__ boff, const uint64_t* __restrict__ qkey,
                                             int64_t g0, uint64_t key, int32_t r, int32_t ge = INT32_MIN) {
    const int32_t g1 = ge != INT32_MIN ? ge : gend[g0];
    if (g1 < 0) return -1;
    const int n = (int)(g1 - g0);
    int lb = 5;
    while ((1 << lb) < (n + 1) / 2) ++lb;
    const uint32_t b = (uint32_t)(key >> (64 - lb));
    const uint32_t lo = boff[g0 + b], hi = boff[g0 + b + 1];
    const uint64_t k48 = key >> 16;
    int32_t cand = -1, m = 0;
    for (uint32_t x = lo; x < hi; ++x) {
        const uint64_t v = gq[g0 + x];
        if ((v >> 16) != k48) continue;
        const int32_t rec = (int32_t)(g0 + (int64_t)(v & 0xffffu));
        // (the entry's 48 key bits and the bucket's top bits are the match; the qnames are compared
        // exactly afterwards, and two records matching here send the read to the exact residual path)
        if (rec != r) { cand = rec; ++m; }
    }
    (void)qkey;
    return m == 1 ? cand : -1;
}

// The global search: the one in-pairing record of the target position group (tid, pos) = target
// with qname key `key` other than record r; -1 when there is none, several, or the group is deeper
// than GRP_SMALL + 1 records (residual).
__device__ __forceinline__ int32_t mate_search_global(int64_t N, const uint64_t* __restrict__ rkey,
                                                      const uint64_t* __restrict__ rq, const DevTable& T,
                                                      int32_t r, int32_t mtid, int32_t mpos, uint64_t target,
                                                      uint64_t key, int64_t hint, const uint64_t* __restrict__ gq,
                                                      const int32_t* __restrict__ gend,
                                                      const uint32_t* __restrict__ boff) {
    // the lower bound of the target is at most `hint` (rkey[hint] >= target): gallop down from it in
    // steps growing 4x, then bisect the last step
    int64_t x = 0;
    {
        int64_t hi = hint, lo = hint;
        for (int64_t step = 256;; step <<= 2) {
            lo = hi - step;
            if (lo <= 0) { lo = 0; break; }
            if (rkey[lo] < target) break;
            hi = lo;
        }
        x = lo;
        while (x < hi) {
            const int64_t mid = (x + hi) >> 1;
            if (rkey[mid] < target) x = mid + 1;
            else hi = mid;
        }
    }
    // a group deeper than GRP_SMALL + 1 is searched by bisection over its sorted keys (deep_find),
    // or goes to the residual when they were not sorted: one probe past its first GRP_SMALL + 1
    // records (x is the group's first record) says so up front
    if (x + GRP_SMALL + 1 < N && rkey[x] == target && rkey[x + GRP_SMALL + 1] == target)
        return gq ? deep_find(gq, gend, boff, rq, x, key, r) : -1;
    // walk 4 records per round (independent loads): skip keys below the target, then the
    // target's position group, at most GRP_SMALL + 1 of it (deeper: residual)
    int32_t cand = -1, m = 0, ng = 0;
    for (bool over = false; !over; x += 4) {
        uint64_t kk[4], qq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            kk[u] = x + u < N ? rkey[x + u] : 0ULL;
            qq[u] = x + u < N ? rq[x + u] : 0ULL;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (over || (x + u < N && kk[u] < target)) continue;
            if (x + u >= N || kk[u] != target) { over = true; continue; }
            if (ng > GRP_SMALL) return -1;                   // (deep groups were taken above)
            ++ng;
            if (x + u != r && qq[u] == key) { cand = (int32_t)(x + u); ++m; }
        }
    }
    return m == 1 ? cand : -1;                               // none or several: residual
}

// The pair (stream entries s and sx) found by s's search: s claims sx, the later end completes it.
__device__ __forceinline__ void mate_record(int64_t s, int32_t sx, uint64_t key, int32_t* __restrict__ partner,
                                            int32_t* __restrict__ claimer, int32_t* __restrict__ mate_of,
                                            uint8_t* __restrict__ pflag, unsigned long long* __restrict__ ltab,
                                            uint64_t lmask, uint32_t& n_long, bool both_search,
                                            uint32_t* __restrict__ err) {
    partner[s] = sx;
    claimer[sx] = (int32_t)s;   // plain store: a second claimer overwrites, k_pair_resid sees it
    const int32_t s1 = (int32_t)s < sx ? (int32_t)s : sx, s2 = (int32_t)s < sx ? sx : (int32_t)s;
    mate_of[s2] = s1;
    pflag[s2] = 1;
    // Two pairs of one qname found here (four occurrences, interleaved in the stream) would pair
    // differently in pair_dict's stream order.  Pairs spanning at most PD_W stream entries are
    // checked tile by tile in LDS (k_pair_resid); the few longer ones (translocations, long inserts)
    // enter their key here in an exact table that the short ones probe.  A long pair has one
    // searcher, except when both ends sit at one position (a deep group): then the later one enters it.
    if (s2 - s1 > PD_W && (!both_search || s == s2)) {
        ++n_long;
        uint64_t h = key & lmask;
        bool done = false;
        for (uint64_t i = 0; i <= lmask && !done; ++i) {
            const unsigned long long prev = atomicCAS(&ltab[h], ~0ULL, key);
            if (prev == ~0ULL) done = true;
            else if (prev == key) { atomicOr(err, EB_NEEDSORT); done = true; }
            else h = (h + 1) & lmask;
        }
        if (!done) atomicOr(err, EB_NEEDSORT);   // table full: the sort path decides
    }
}

// The same search on an identity stream (the table itself, stream entry = record) with the keys
// staged in LDS: a block takes TILE entries and stages the record keys and qname keys of the
// PC_HALO entries before them (mates lie at or before the searcher) and GRP_SMALL + 2 after (a
// position group running past the searcher).  A target group found whole inside the staged range
// is walked there; one that may begin before it (or end after it) takes the global search.
// TILE 1024 on large tables; 512 below PC_SMALL_N records, where the launch is one round of blocks
// and each block's latency chain is the kernel's time (twice the blocks, half the entries per thread)
constexpr int PC_HALO = 512;
constexpr int64_t PC_SMALL_N = (int64_t)1 << 23;
template <int TILE>
__global__ __launch_bounds__(256) void k_pair_coord_tile(int64_t N, const uint64_t* __restrict__ skey,
                                                         const int32_t* __restrict__ spos,
                                                         const uint64_t* __restrict__ rkey, DevTable T,
                                                         int32_t* __restrict__ partner, int32_t* __restrict__ claimer,
                                                         int32_t* __restrict__ mate_of, uint8_t* __restrict__ pflag,
                                                         unsigned long long* __restrict__ ltab, uint64_t lmask,
                                                         uint32_t* __restrict__ long_stripes, uint32_t* __restrict__ err,
                                                         const uint64_t* __restrict__ gq, const int32_t* __restrict__ gend,
                                                         const uint32_t* __restrict__ boff,
                                                         const unsigned long long* __restrict__ dgk, uint64_t dgmask) {
    __shared__ uint64_t s_k[(TILE + PC_HALO + GRP_SMALL + 2)], s_q[(TILE + PC_HALO + GRP_SMALL + 2)];
    const int64_t t0 = xcd_block() * TILE;
    const int64_t t1 = min(N, t0 + TILE);
    const int64_t w0 = t0 > PC_HALO ? t0 - PC_HALO : 0;
    const int64_t w1 = min(N, t1 + GRP_SMALL + 2);
    const int nw = (int)(w1 - w0);
    // the own entries' mate coordinates, loaded alongside the staging
    int32_t mt[TILE / 256], mp[TILE / 256];
#pragma unroll
    for (int u = 0; u < TILE / 256; ++u) {
        const int64_t s = t0 + threadIdx.x + 256 * u;
        mt[u] = s < t1 ? T.mtid[s] : 0;
        mp[u] = s < t1 ? T.mpos[s] : 0;
    }
    for (int i = threadIdx.x; i < nw; i += blockDim.x) {
        s_k[i] = rkey[w0 + i];
        s_q[i] = skey[w0 + i];
    }
    __syncthreads();
    // Each thread takes PC_PER entries (blockDim apart) in phases, so that the global loads of its
    // entries are in flight together: the searches in LDS, then the candidates' qnames, then the
    // stores.
    constexpr int PC_PER = TILE / 256;
    int32_t cand[PC_PER];
    uint64_t key[PC_PER], tgt[PC_PER];
#pragma unroll
    for (int u = 0; u < PC_PER; ++u) {
        const int64_t s = t0 + threadIdx.x + 256 * u;
        cand[u] = -1;
        key[u] = ~0ULL;
        tgt[u] = ~0ULL;
        if (s >= t1) continue;
        const int li = (int)(s - w0);
        key[u] = s_q[li];
        if (!spos) partner[s] = -1;                          // mate_record overwrites a found mate's
        if (key[u] == ~0ULL) continue;
        const int32_t r = (int32_t)s;
        const int32_t mtid = mt[u], mpos = mp[u];
        const uint64_t target = pos_key(mtid, mpos);
        tgt[u] = target;
        if (target > s_k[li]) continue;                      // the mate searches (or is elsewhere)
        if (dgk) {
            // a deep target group (listed by k_build_meta): bisection over its sorted qname keys
            const int2 dg = dg_lookup(dgk, dgmask, target);
            if (dg.x >= 0) {
                cand[u] = deep_find(gq, gend, boff, skey, dg.x, key[u], r, dg.y);
                continue;
            }
        }
        // lower_bound(target) in the staged keys; s_k[li] >= target, so it is at most li
        int lo = 0, hi = li;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_k[mid] < target) lo = mid + 1;
            else hi = mid;
        }
        if (lo == 0 && w0 > 0) {
            // the group may begin before the staged range: the table is searched from there (a deep
            // group by bisection over its sorted keys, or residual when they were not sorted)
            int x = 0;
            while (x < nw && x <= GRP_SMALL + 1 && s_k[x] == target) ++x;
            cand[u] = x > GRP_SMALL + 1 && !gq ? -1
                      : mate_search_global(N, rkey, skey, T, r, mtid, mpos, target, key[u], w0, gq, gend, boff);
        } else {
            int x = lo, ng = 0, m = 0, c = -1;
            bool deep = false;
            for (; x < nw && s_k[x] == target; ++x) {
                if (ng > GRP_SMALL) { deep = true; break; }
                ++ng;
                if (x != li && s_q[x] == key[u]) { c = (int32_t)(w0 + x); ++m; }
            }
            if (deep) c = gq ? deep_find(gq, gend, boff, skey, w0 + lo, key[u], r) : -1;   // the group starts at w0 + lo
            else if (x == nw && w1 < N)   // the group runs past the staged range: its start is known
                c = mate_search_global(N, rkey, skey, T, r, mtid, mpos, target, key[u], w0 + lo, gq, gend, boff);
            else if (m != 1) c = -1;
            cand[u] = c;
        }
    }
    // the qnames of every found candidate pair, their words loaded together
    bool ok[PC_PER];
    {
        int la[PC_PER], lb[PC_PER];
        const uint64_t* wa[PC_PER];
        const uint64_t* wb[PC_PER];
#pragma unroll
        for (int u = 0; u < PC_PER; ++u) {
            const int32_t r = (int32_t)(t0 + threadIdx.x + 256 * u), c = cand[u] < 0 ? r : cand[u];
            const bool f = cand[u] >= 0;
            const uint64_t oa = f ? T.qn_ol[r] : 0ULL, ob = f ? T.qn_ol[c] : 0ULL;   // one word each
            la[u] = (int)(oa & 0xffffu);
            lb[u] = (int)(ob & 0xffffu);
            wa[u] = reinterpret_cast<const uint64_t*>(T.qn_blob + (oa >> 16));
            wb[u] = reinterpret_cast<const uint64_t*>(T.qn_blob + (ob >> 16));
        }
#pragma unroll
        for (int u = 0; u < PC_PER; ++u) {
            const int nw8 = (la[u] + 7) >> 3;
            uint64_t d = la[u] != lb[u] ? 1ULL : 0ULL;
#pragma unroll
            for (int w = 0; w < 4; ++w)
                if (w < nw8) d |= wa[u][w] ^ wb[u][w];
            for (int w = 4; w < nw8 && !d; ++w) d |= wa[u][w] ^ wb[u][w];
            ok[u] = cand[u] >= 0 && d == 0;
        }
    }
    uint32_t nl = 0;
#pragma unroll
    for (int u = 0; u < PC_PER; ++u)
        if (ok[u]) {
            // stream entries: the records themselves on an identity stream, else their stream slots
            const int32_t r = (int32_t)(t0 + threadIdx.x + 256 * u);
            // both ends search when they sit at one position (the mate's key equals the own)
            const bool both = tgt[u] == rkey[r];   // (the candidate lies in the target position group)
            mate_record(spos ? spos[r] : r, spos ? spos[cand[u]] : cand[u], key[u], partner, claimer, mate_of, pflag,
                        ltab, lmask, nl, both, err);
        }
    stripe_add(nl, long_stripes);
}

// After the mate search, per tile of PD_TILE stream entries (one block):
//  * inconsistencies only pair_dict's stream order can settle (a qname seen more than twice):
//    a read claimed by two searchers, a found mate that found another read, a searcher claimed by
//    a third read -> EB_NEEDSORT (the pass re-runs on the sort path);
//  * one qname in two found pairs, exactly: two such pairs interleave in the stream only if each
//    holds an end inside the other's span, so with spans of at most PD_W entries their later ends
//    lie within PD_W of each other.  The block enters every found pair with an end in its tile or
//    the PD_W entries before it in an LDS table as (key fingerprint, later end); the same key
//    (compared in full through the entered end's stream key) with another later end is a qname
//    paired twice.  Pairs longer than PD_W were entered in the global table by the mate search; the
//    short pairs ending in the tile probe it when it is not empty;
//  * unpaired and unclaimed entries are residual (the exact sort path pairs them).
__global__ __launch_bounds__(256) void k_pair_resid(int64_t S, const uint64_t* __restrict__ skey,
                                                    const int32_t* __restrict__ partner,
                                                    const int32_t* __restrict__ claimer, uint8_t* __restrict__ resid,
                                                    uint32_t* __restrict__ n_resid,
                                                    const unsigned long long* __restrict__ ltab, uint64_t lmask,
                                                    const uint32_t* __restrict__ n_long, uint32_t* __restrict__ err) {
    __shared__ uint32_t s_tab[PD_SLOTS];
    const int t = threadIdx.x;
    const int64_t t0 = (int64_t)blockIdx.x * PD_TILE, t1 = min(S, t0 + PD_TILE);
    const int64_t base = max((int64_t)0, t0 - PD_W);
    for (int i = t; i < PD_SLOTS; i += blockDim.x) s_tab[i] = ~0u;
    __syncthreads();
    const bool any_long = *n_long != 0u;
    uint32_t eb = 0, nres = 0;
    for (int64_t x = base + t; x < t1; x += blockDim.x) {
        const uint64_t key = skey[x];
        const int32_t px = partner[x];
        const int32_t cl = claimer[x];
        if (x >= t0) {
            uint32_t rs = 0;
            if (key != ~0ULL) {
                if (px >= 0) {
                    if (claimer[px] != (int32_t)x) eb |= EB_NEEDSORT;   // px claimed twice
                    const int32_t pp = partner[px];
                    if ((pp >= 0 || cl >= 0) && pp != (int32_t)x) eb |= EB_NEEDSORT;
                }
                rs = (px < 0 && cl < 0) ? 1u : 0u;
            }
            resid[x] = (uint8_t)rs;
            nres += rs;
        }
        const int32_t other = px >= 0 ? px : cl;
        if (other < 0) continue;
        const int32_t lo = (int32_t)x < other ? (int32_t)x : other, hi = (int32_t)x < other ? other : (int32_t)x;
        if (hi - lo > PD_W) continue;                       // long pair: the global table has it
        if (x == hi && x >= t0 && any_long) {               // probe the long pairs' keys
            uint64_t h = key & lmask;
            for (uint64_t i = 0; i <= lmask; ++i) {
                const unsigned long long k = ltab[h];
                if (k == ~0ULL) break;
                if (k == key) { eb |= EB_NEEDSORT; break; }
                h = (h + 1) & lmask;
            }
        }
        const uint32_t fp = (uint32_t)(key >> 44);
        const uint32_t ent = (fp << 12) | (uint32_t)(hi - base);
        uint32_t slot = (uint32_t)(key >> 11) & (PD_SLOTS - 1);
        bool done = false;
        for (int i = 0; i < PD_SLOTS && !done; ++i) {
            const uint32_t prev = atomicCAS(&s_tab[slot], ~0u, ent);
            if (prev == ~0u || prev == ent) {
                done = true;                                  // entered, or the same pair's other end
            } else if ((prev >> 12) == fp && skey[base + (prev & 0xfffu)] == key) {
                eb |= EB_NEEDSORT;                            // the same qname, another pair
                done = true;
            } else {
                slot = (slot + 1) & (PD_SLOTS - 1);
            }
        }
        if (!done) eb |= EB_NEEDSORT;
    }
    stripe_add(nres, n_resid);
    if (eb) atomicOr(err, eb);
}

// The residual keys (stream entries the coordinate search left unpaired), compacted in the scan of
// their byte flags (EmitResid): the sort's input, and for the probe below an exact table of the keys
// behind a blocked Bloom filter (one 64-bit word per key, 3 bits set in it; 16 bits per key, so the
// filter stays in L2 / the MALL and a paired entry touches the table only on a filter hit).
__device__ __forceinline__ uint64_t bloom_bits(uint64_t k) {
    return (1ULL << (k & 63)) | (1ULL << ((k >> 6) & 63)) | (1ULL << ((k >> 12) & 63));
}
__device__ __forceinline__ uint64_t bloom_word(uint64_t k, uint64_t bmask) { return (k >> 24) & bmask; }

struct EmitResid {   // residual entries (byte flags): key and stream slot compacted, table and filter
    static constexpr bool kPlain = false;
    const uint64_t* skey;
    uint64_t* rk;
    uint32_t* rv;
    int64_t cap;        // a planned re-run's residual count: more re-run the pass exactly (EB_PLAN)
    unsigned long long* ht;   // null: many residual reads, the sorted keys are searched instead
    uint64_t hmask;
    unsigned long long* bloom;
    uint64_t bmask;
    uint32_t* err;
    // per table slot: occurrences, first and last stream slot (k_resid_pair pairs a key seen twice
    // without the sort); n_multi counts keys seen three times or more (those take the sort path)
    uint32_t *hcnt, *hmin, *hmax, *n_multi;
    __device__ void operator()(int64_t i, uint32_t x, uint32_t f) const {
        if (!f) return;
        if ((int64_t)x >= cap) { atomicOr(err, EB_PLAN); return; }
        const uint64_t k = skey[i];
        rk[x] = k;
        rv[x] = (uint32_t)i;
        if (!ht) return;
        atomicOr(&bloom[bloom_word(k, bmask)], (unsigned long long)bloom_bits(k));
        uint64_t slot = k & hmask;
        for (uint64_t p = 0; p <= hmask; ++p) {
            const unsigned long long prev = atomicCAS(&ht[slot], ~0ULL, k);
            if (prev == ~0ULL || prev == k) {
                if (atomicAdd(&hcnt[slot], 1u) == 2u) atomicAdd(n_multi, 1u);
                atomicMin(&hmin[slot], (uint32_t)i);
                atomicMax(&hmax[slot], (uint32_t)i);
                return;
            }
            slot = (slot + 1) & hmask;
        }
        atomicOr(err, EB_PLAN);   // table full
    }
};

// k_pair_mark's pairing of the residual reads when no key occurs three times or more: a key seen
// twice pairs its later occurrence with its earlier one (qnames compared), a key seen once is an
// unpaired read; no sort
__global__ __launch_bounds__(256) void k_resid_pair(int64_t NR, const uint64_t* __restrict__ rk,
                                                    const uint32_t* __restrict__ rv,
                                                    const unsigned long long* __restrict__ ht, uint64_t hmask,
                                                    const uint32_t* __restrict__ hcnt, const uint32_t* __restrict__ hmin,
                                                    const uint32_t* __restrict__ hmax, int ident,
                                                    const int32_t* __restrict__ stream_rec, DevTable T,
                                                    int32_t* __restrict__ mate_of, uint8_t* __restrict__ pflag,
                                                    uint32_t* __restrict__ err, unsigned long long* __restrict__ cnt) {
    int acc[1] = {0};
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < NR) {
        const uint64_t k = rk[x];
        const uint32_t i = rv[x];
        uint64_t slot = k & hmask;
        for (uint64_t p = 0; p <= hmask && ht[slot] != k; ++p) slot = (slot + 1) & hmask;
        const uint32_t c = hcnt[slot];
        if (c == 1u) acc[0] = 1;
        else if (c == 2u) {
            if (i == hmax[slot]) {
                const uint32_t a = hmin[slot];
                if (qname_eq(T, ident ? (int32_t)a : stream_rec[a], ident ? (int32_t)i : stream_rec[i])) {
                    mate_of[i] = (int32_t)a;
                    pflag[i] = 1;
                } else {
                    atomicOr(err, EB_COLLISION);
                }
            }
        } else {
            atomicOr(err, EB_PLAN);   // a key seen 3+ times on a pass planned without any: re-run exactly
        }
    }
    const int slots[1] = {CC_CNT_UNPAIRED};
    block_count<1>(acc, slots, cnt);
}

// a qname key paired by coordinates must not also occur among the residual reads (3+ occurrences:
// the pass re-runs on the sort path)
__global__ __launch_bounds__(256) void k_resid_probe(int64_t S, const uint64_t* __restrict__ skey,
                                                     const uint8_t* __restrict__ resid,
                                                     const unsigned long long* __restrict__ ht, uint64_t mask,
                                                     const unsigned long long* __restrict__ bloom, uint64_t bmask,
                                                     uint32_t* __restrict__ err) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const uint64_t k = skey[s];
    if (k == ~0ULL || resid[s]) return;
    const uint64_t bb = bloom_bits(k);
    if ((bloom[bloom_word(k, bmask)] & bb) != bb) return;
    uint64_t slot = k & mask;
    for (uint64_t i = 0; i <= mask; ++i) {
        const unsigned long long h = ht[slot];
        if (h == ~0ULL) break;
        if (h == k) { atomicOr(err, EB_NEEDSORT); break; }
        slot = (slot + 1) & mask;
    }
}

// the same check against the sorted residual keys (binary search), for passes where most reads
// are residual (deep position groups, c4) and a hash table of all of them would cost one scattered
// atomic per read
__global__ __launch_bounds__(256) void k_resid_probe_sorted(int64_t S, const uint64_t* __restrict__ skey,
                                                            const uint8_t* __restrict__ resid,
                                                            const uint64_t* __restrict__ sorted, int64_t nr,
                                                            uint32_t* __restrict__ err) {
    int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const uint64_t k = skey[s];
    if (k == ~0ULL || resid[s]) return;
    int64_t lo = 0, hi = nr;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (sorted[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    if (lo < nr && sorted[lo] == k) atomicOr(err, EB_NEEDSORT);
}


// Per completed pair (records from the pair scan, EmitPairs): the consensus key's hash (csn_pair_dict)
// and both ends' unique_tag hashes (read_dict / tag_dict grouping); tags and keys themselves are
// recomputed from the records where they are compared (make_tag / make_ckey).
__global__ __launch_bounds__(256) void k_pair_keys(int64_t P, PairView V, DevTable T, uint64_t seed,
                                                   uint64_t* __restrict__ chash, uint64_t* __restrict__ thash,
                                                   uint32_t* __restrict__ tval, int4* __restrict__ ptag,
                                                   uint64_t* __restrict__ rec_hash) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const int32_t a = V.rec1[p], b = V.rec2[p];
    const uint32_t run = pair_run(V, (int32_t)p);
    const RecCore A = T.core[CC_IDX(a, T.n, DS_REC)], B = T.core[CC_IDX(b, T.n, DS_REC)];
    const CKey c = make_ckey_c(A, B, run);
    const TagKey t0 = make_tag_c(A, B, 0, run), t1 = make_tag_c(A, B, 1, run);
    chash[p] = hash_ckey(c, seed);
    const int4 pt = make_int4(t0.bc, t0.cigA, t0.cigB, (int32_t)run);
    if (rec_hash) {   // sorted table: by record, read coalesced by the position-group ranking
        rec_hash[a] = hash_tag(t0, seed);
        rec_hash[b] = hash_tag(t1, seed);
    } else {          // sort path: by read end, the tag sort's keys
        thash[2 * p] = hash_tag(t0, seed);
        thash[2 * p + 1] = hash_tag(t1, seed);
    }
    if (tval) { tval[2 * p] = (uint32_t)(2 * p); tval[2 * p + 1] = (uint32_t)(2 * p + 1); }   // sort path only
    ptag[p] = pt;
}

// Per member (sorted read-end j) a 16-byte record the votes read in one coalesced load:
//   x = payload offset / 16, y = tlen, z = lseq | qlen << 16 (0xffff: no cigar),
//   w = flag (12b) | mapq << 12 | rflags(3b) << 20 | valid << 23 | rg7 << 24
//       (rg7 0x7f: no RG, 0x7e: id >= 126, look it up)
__device__ __forceinline__ uint4 pack_meta(const DevTable& T, int32_t r, bool valid) {
    uint4 m = T.meta[CC_IDX(r, T.n, DS_MEMBER)];   // k_build_meta
    m.w |= (valid ? 1u : 0u) << 23;
    return m;
}

// mem_rec[j] for j < n_known was written by k_group_rank (the record of the ranked end)
__global__ __launch_bounds__(256) void k_fam_mark(int64_t R, int64_t n_known, int64_t j0,
                                                  const uint64_t* __restrict__ rs_key,
                                                  const uint32_t* __restrict__ rs_val, PairView V, DevTable T,
                                                  uint8_t* __restrict__ segf, uint32_t* __restrict__ validf,
                                                  int32_t* __restrict__ mem_rec, uint4* __restrict__ mem_meta,
                                                  uint32_t* __restrict__ err, int same_grp) {
    // same_grp: equal keys imply one position group (group-major deep keys), so the tag compare
    // skips (tid, pos), which agree by construction
    const int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = j < R;
    const int lane = threadIdx.x & 63;
    const uint32_t e = in ? rs_val[j] : 0u;
    int32_t r = 0;
    if (in) r = j < n_known ? mem_rec[j] : ((e & 1) ? V.rec2[e >> 1] : V.rec1[e >> 1]);
    // each slot's tag (gathered once) goes to the next lane: the equal-hash comparison with the
    // previous slot reads one tag per slot instead of two (lane 0 gathers its previous slot's)
    const TagKey mine = !in ? TagKey{} : same_grp ? tag_of_rec_np(T, r, V.tag[e >> 1]) : tag_of_rec(T, r, V.tag[e >> 1]);
    TagKey prevt;
    {
        const int32_t* m = reinterpret_cast<const int32_t*>(&mine);
        int32_t* p = reinterpret_cast<int32_t*>(&prevt);
#pragma unroll
        for (int k = 0; k < 8; ++k) p[k] = __shfl(m[k], (lane + 63) & 63, 64);
    }
    if (!in) return;
    // the first slot of the range starts a family (j0 = n_known: the deep groups' ends, whose
    // positions no small group's end shares)
    bool start = (j == j0) || rs_key[j - 1] != rs_key[j];
    const uint32_t prev = j > 0 ? rs_val[j - 1] : 0;
    if (!start) {
        if (lane == 0) {
            const int32_t pr = (j - 1 < n_known) ? mem_rec[j - 1] : ((prev & 1) ? V.rec2[prev >> 1] : V.rec1[prev >> 1]);
            prevt = same_grp ? tag_of_rec_np(T, pr, V.tag[prev >> 1]) : tag_of_rec(T, pr, V.tag[prev >> 1]);
        }
        if (!tag_eq(mine, prevt)) {
            atomicOr(err, EB_COLLISION);
            start = true;
        }
    }
    const bool valid = start || ((e >> 1) != (prev >> 1));
    segf[j] = start ? 1 : 0;
    validf[j] = valid;
    if (j >= n_known) mem_rec[j] = r;
    if (mem_meta) mem_meta[j] = pack_meta(T, r, valid);
}

// The member records of a grouping whose pass did not write them (only passes that list bad reads,
// the SSCS stage's, write them as they rank; another caller's vote builds them here)
__global__ __launch_bounds__(256) void k_mem_meta(int64_t R, const int32_t* __restrict__ mem_rec,
                                                  const uint32_t* __restrict__ validf, DevTable T,
                                                  uint4* __restrict__ mem_meta) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < R) mem_meta[j] = pack_meta(T, mem_rec[j], validf[j] != 0u);
}

// "line read twice" in general (consensus_helper.py:490-500): read end j joins its family only if
// the first read of its pair (pair_dict[qname][0]) is not already a member, by record equality
// (pysam __eq__, here the records' byte digests).  k_fam_mark applies the rule in its usual form
// (the previous member comes from the same pair); when a qname was seen more than twice, equal
// records can sit in different pairs, and this pass re-decides every family serially in member
// (completion) order.  One thread per family; early exit when no qname was seen more than twice.
__global__ __launch_bounds__(256) void k_fam_dedup(int64_t R, const uint32_t* __restrict__ n_multi,
                                                   const uint8_t* __restrict__ segf, uint32_t* __restrict__ validf,
                                                   const int32_t* __restrict__ mem_rec,
                                                   const uint32_t* __restrict__ rs_val,
                                                   const int32_t* __restrict__ pr_rec1, const uint64_t* __restrict__ rdig,
                                                   uint4* __restrict__ mem_meta) {
    if (*n_multi == 0) return;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < R; j += stride) {
        if (!segf[j]) continue;
        for (int64_t k = j + 1; k < R && !segf[k]; ++k) {
            const uint64_t first = rdig[pr_rec1[rs_val[k] >> 1]];
            bool in = false;
            for (int64_t m = j; m < k && !in; ++m) in = validf[m] && rdig[mem_rec[m]] == first;
            validf[k] = in ? 0u : 1u;
            if (!mem_meta) continue;
            uint4 mm = mem_meta[k];
            mm.w = (mm.w & ~(1u << 23)) | ((in ? 0u : 1u) << 23);
            mem_meta[k] = mm;
        }
    }
}

// ---- tag grouping by position groups (coordinate-sorted tables) ---------------------------
// unique_tag includes the read's own (tid, pos) (consensus_helper.py:295-304), so all members of
// a family lie in one group of equal (tid, pos) in a coordinate-sorted table.  Inside each group
// of at most GRP_SMALL records the read ends are ranked by (tag hash, completion index): that
// places families contiguously with members in pair-completion order, without a global sort.


// Records are processed in tiles of GT staged in LDS with GH = GRP_SMALL records of halo on each
// side.  The staged keys become head bits (a group starts here; entries outside [lo, hi) and the
// first staged entry count as heads), so a record's group is [highest head <= it, lowest head
// > it): a clz/ffs over at most three words.  A group that reaches the staged edge has spanned
// more than GRP_SMALL records (deep), so nothing is looked up outside LDS.
constexpr int GT = 256, GH = GRP_SMALL, GS = GT + 2 * GH, GW = GS / 32;

__device__ __forceinline__ void tile_range(int64_t N, int64_t b0, int nt, int& lo, int& hi) {
    lo = b0 >= GH ? 0 : (int)(GH - b0);
    const int64_t after = N - b0 - nt;
    hi = GH + nt + (int)(after < GH ? after : GH);
}

// head bits of the staged keys (s_k filled for [lo, hi) and synchronised); every wave takes part
__device__ __forceinline__ void tile_heads(const uint64_t* s_k, int lo, int hi, uint32_t* s_hd) {
    for (int i = threadIdx.x; i < GS; i += GT) {
        const bool hd = i <= lo || i >= hi || s_k[i] != s_k[i - 1];
        const uint64_t m = __ballot(hd);
        if ((threadIdx.x & 63) == 0) {
            s_hd[i >> 5] = (uint32_t)m;
            s_hd[(i >> 5) + 1] = (uint32_t)(m >> 32);
        }
    }
}

__device__ __forceinline__ void tile_span(const uint32_t* s_hd, int li, int& a, int& z) {
    int w = li >> 5;
    uint32_t m = s_hd[w] & (0xffffffffu >> (31 - (li & 31)));
    while (!m) m = s_hd[--w];                       // entry 0 is a head
    a = 32 * w + 31 - __clz(m);
    const int i = li + 1;
    z = GS;
    if (i < GS) {
        w = i >> 5;
        m = s_hd[w] & (0xffffffffu << (i & 31));
        while (!m && ++w < GW) m = s_hd[w];
        if (m) z = 32 * w + __ffs(m) - 1;
    }
}

// per tile of GT records: the read ends in groups of at most GRP_SMALL records (ranked in place by
// k_group_rank, which takes its tile's first slot from the scan of these counts); read ends of
// deeper groups are flagged for the sort path
__global__ __launch_bounds__(GT) void k_group_flags(int64_t N, const uint64_t* __restrict__ rkey,
                                                    const int32_t* __restrict__ rec_e, uint32_t* __restrict__ tile_small,
                                                    uint32_t* __restrict__ bigE, uint32_t* __restrict__ n_big) {
    __shared__ uint32_t s_c[GT / 64];
    __shared__ uint64_t s_k[GS];
    __shared__ uint32_t s_hd[GW];
    const int64_t b0 = xcd_block() * GT;
    const int t = threadIdx.x;
    const int nt = (int)(N - b0 < GT ? N - b0 : GT);
    int lo, hi;
    tile_range(N, b0, nt, lo, hi);
    for (int i = t; i < GS; i += GT)
        if (i >= lo && i < hi) s_k[i] = rkey[b0 - GH + i];
    __syncthreads();
    tile_heads(s_k, lo, hi, s_hd);
    __syncthreads();
    uint32_t big = 0, sm = 0;
    if (t < nt) {
        const int64_t r = b0 + t;
        const int32_t e = rec_e[r];
        if (e >= 0) {
            int a, z;
            tile_span(s_hd, t + GH, a, z);
            if (z - a <= GRP_SMALL) sm = 1u;
            else { bigE[e] = 1u; big = 1u; }
        }
    }
    stripe_add(big, n_big);
    const uint64_t m = __ballot(sm != 0u);
    if ((t & 63) == 0) s_c[t >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    if (t == 0) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < GT / 64; ++w) c += s_c[w];
        tile_small[b0 / GT] = c;
    }
}

// A small group's read ends by (tag hash, end index): end r goes to cp(r) - (ends of its group
// before it) + rank, i.e. its group's first compacted slot plus its rank, where cp(r) counts the
// small groups' ends before record r (the tile's scanned count plus the block's own).  The family marks of
// k_fam_mark are settled here too, for the small groups' slots: a slot starts a family unless the
// end ranked just before it in its group has the same hash (then the tags are compared field by
// field: a 64-bit collision is EB_COLLISION); it is valid unless that end is its own pair's other
// end ("line read twice"); and its 16-B member record is the record's (read coalesced here).
__global__ __launch_bounds__(GT) void k_group_rank(int64_t N, const uint64_t* __restrict__ rkey,
                                                   const int32_t* __restrict__ rec_e, const uint64_t* __restrict__ rhash,
                                                   const uint32_t* __restrict__ tile_pre,
                                                   uint64_t* __restrict__ rs_key, uint32_t* __restrict__ rs_val,
                                                   int32_t* __restrict__ rs_rec, PairView V,
                                                   DevTable T, uint8_t* __restrict__ segf, uint32_t* __restrict__ validf,
                                                   uint4* __restrict__ mem_meta, uint32_t* __restrict__ err) {
    __shared__ uint64_t s_k[GS], s_h[GS];
    __shared__ int32_t s_e[GS];
    __shared__ uint32_t s_hd[GW];
    __shared__ uint32_t s_c[GT / 64];
    const int64_t b0 = xcd_block() * GT;
    const int t = threadIdx.x;
    const int nt = (int)(N - b0 < GT ? N - b0 : GT);
    const uint32_t base = tile_pre[b0 / GT];   // the tile's first compacted slot (scan of k_group_flags' counts)
    int lo, hi;
    tile_range(N, b0, nt, lo, hi);
    for (int i = t; i < GS; i += GT) {
        if (i < lo || i >= hi) continue;
        const int64_t rr = b0 - GH + i;
        s_k[i] = rkey[rr];
        s_e[i] = rec_e[rr];
        s_h[i] = rhash[rr];   // meaningful where the record has a read end (s_e >= 0)
    }
    __syncthreads();
    tile_heads(s_k, lo, hi, s_hd);
    __syncthreads();
    const int32_t r = (int32_t)(b0 + t);
    const int li = t + GH;
    int a = 0, z = 0;
    bool sm = false;
    if (t < nt && s_e[li] >= 0) {
        tile_span(s_hd, li, a, z);
        sm = z - a <= GRP_SMALL;
    }
    // the record's compacted slot among the small groups' ends: the tile's base plus the block's
    // exclusive count before it (k_group_flags counted the same flags)
    const uint64_t bm = __ballot(sm);
    const int lane = t & 63;
    if (lane == 0) s_c[t >> 6] = (uint32_t)__popcll(bm);
    __syncthreads();
    if (!sm) return;
    // the record's own fields for the tag compare and its member record, loaded ahead of the walk
    const int fo = T.flag[r];
    const int32_t omt = T.mtid[r], omp = T.mpos[r];
    const uint4 om = mem_meta ? T.meta[CC_IDX(r, T.n, DS_MEMBER)] : make_uint4(0u, 0u, 0u, 0u);
    uint32_t cpv = base + (uint32_t)__popcll(bm & ((1ULL << lane) - 1ULL));
    for (int w = 0; w < (t >> 6); ++w) cpv += s_c[w];
    const int32_t e = s_e[li];
    const uint64_t h = s_h[li];
    uint32_t before = 0, rank = 0;
    int32_t pe = -1, pj = 0;    // the end ranked just before this one in the group, and its tile slot
    uint64_t ph = 0;
    for (int j = a; j < z; ++j) {
        const int32_t ej = s_e[j];
        if (ej < 0) continue;
        const uint64_t hj = s_h[j];
        before += j < li ? 1u : 0u;
        if (hj < h || (hj == h && ej < e)) {
            ++rank;
            if (pe < 0 || hj > ph || (hj == ph && ej > pe)) { pe = ej; ph = hj; pj = j; }
        }
    }
    const uint32_t o = CC_IDX(cpv - before + rank, N, DS_SLOT);
    bool start = pe < 0 || ph != h;
    // equal hashes: the exact tags (unique_tag, consensus_helper.py:295-304).  Both ends sit in this
    // position group, so tid and pos agree; the rest is the pair's shared fields {bc, cigA, cigB,
    // run}, the end's mate coordinates and its orientation / read number flag bits.
    if (!start) {
        const int32_t rp = (int32_t)(b0 - GH + pj);
        const int4 pt = V.tag[e >> 1], pq = V.tag[pe >> 1];
        const int fp = T.flag[rp];
        const bool same = pt.x == pq.x && pt.y == pq.y && pt.z == pq.z && pt.w == pq.w && omt == T.mtid[rp] &&
                          omp == T.mpos[rp] && ((fo >> 4) & 1) == ((fp >> 4) & 1) && which_read(fo) == which_read(fp);
        if (!same) {
            atomicOr(err, EB_COLLISION);
            start = true;
        }
    }
    const bool valid = start || ((e >> 1) != (pe >> 1));
    if (start) rs_key[o] = h;   // read at family starts only (k_fam_build's fam_hash)
    rs_val[o] = (uint32_t)e;
    rs_rec[o] = r;
    segf[o] = start ? 1 : 0;
    validf[o] = valid ? 1u : 0u;
    if (mem_meta) {
        uint4 m = om;
        m.w |= (valid ? 1u : 0u) << 23;
        mem_meta[o] = m;
    }
}

// the deep groups' read ends and their sort keys: the tag hash, or with the records' deep group ids
// (gid, gbits wide) group-major: (gid << (kb - gbits)) | the upper kb - gbits hash bits, kb = 64 or
// 48 (the sort then takes bits 0..kb-1: fewer radix passes at 48), so each group's families come
// out side by side and the family marks read records of one position group together
__global__ __launch_bounds__(256) void k_big_keys(int64_t R, const uint32_t* __restrict__ bigE,
                                                  const uint32_t* __restrict__ bx, const uint64_t* __restrict__ rhash,
                                                  PairView V, const uint32_t* __restrict__ gid, int gbits, int kb,
                                                  uint64_t* __restrict__ bkey, uint32_t* __restrict__ bval) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= R || !bigE[e]) return;
    const int32_t r = (e & 1) ? V.rec2[e >> 1] : V.rec1[e >> 1];
    const uint64_t h = rhash[r];
    bkey[bx[e]] = gid ? (((uint64_t)gid[r] << (kb - gbits)) | (h >> (64 - kb + gbits))) : h;
    bval[bx[e]] = (uint32_t)e;
}

// Deep position groups ranked inside the group, with no global sort (round 4), in three kernels:
//  * k_deep_fam, one 512-thread block per deep group (k_deep_qsort's dlist / gend): the group's read
//    ends go into an LDS table by tag hash (a family per distinct hash, its representative the lowest
//    record), families are numbered in representative order, and each end is placed at its family's
//    offset inside the group's own record range of the scratch `se`, in record order (a sub-round of
//    512 records places wave w's ends of a family after waves 0..w-1's).  The lanes of a wave that
//    share a hash are served by one leader lane (one set of LDS atomics per hash and wave, not one per
//    end: a family's ends otherwise all hit one LDS word); every end's tag is compared field by field
//    with its leader's, each leader's with the representative's (a 64-bit collision is EB_COLLISION,
//    as in k_fam_mark).  Each family becomes a work item {se offset, size, output slot}.
//  * k_deep_emit, one wave per family of up to 64 ends: writes k_fam_mark's slots (end, record,
//    family start, "line read twice" validity, member record), the ends sorted in the wave's
//    registers unless record order is already end order (a coordinate-sorted file whose ties keep
//    the input's pair order: samtools' stable sort of name-grouped aligner output).
//  * k_deep_sortfam, one block per longer family: a family's pairs complete at one position group,
//    so its ends lie close together in end order, and a bitmap over [min, max] in LDS ranks them:
//    an end's slot is the count of set bits below its own (ends are distinct), and an odd end whose
//    bit below is set is its pair's second end in the family ("line read twice").  Families whose
//    ends spread further than the bitmap are merge-sorted in LDS instead (runs of 64 sorted per wave,
//    merged pairwise, each value's place by a branch-free binary search in the other run).
// A group with more than DF_FAMS families or a full table adds to *ovf and writes nothing (the pass
// then takes the sorted path, which rewrites every deep slot); a family longer than DF_SORT sets
// EB_DEEPSORT (the pass re-runs with the group's deep ends on the sorted path).
constexpr int DF_T = 512, DF_SLOTS = 1024, DF_FAMS = 512, DF_SORT = 8192, DF_ST = 512;
constexpr unsigned long long DF_EMPTY = ~0ULL;   // rec_thash values are clamp_key'd: never ~0

__device__ __forceinline__ uint32_t df_slot0(uint64_t h) { return (uint32_t)(h ^ (h >> 31)) & (DF_SLOTS - 1); }
__device__ __forceinline__ int df_find(const unsigned long long* s_key, uint64_t h) {
    uint32_t s = df_slot0(h);
    for (int p = 0; p < DF_SLOTS; ++p) {
        const unsigned long long k = s_key[s];
        if (k == h) return (int)s;
        if (k == DF_EMPTY) return -1;
        s = (s + 1) & (DF_SLOTS - 1);
    }
    return -1;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ TagKey shfl_tag(const TagKey& t, int src) {
    TagKey o;
    const int32_t* m = reinterpret_cast<const int32_t*>(&t);
    int32_t* p = reinterpret_cast<int32_t*>(&o);
#pragma unroll
    for (int k = 0; k < 8; ++k) p[k] = __shfl(m[k], src, 64);
    return o;
}
// ascending bitonic sort of one value per lane over the wave
__device__ __forceinline__ uint32_t wave_sort(uint32_t v, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint32_t u = (uint32_t)__shfl_xor((int)v, j, 64);
            v = (((lane & j) == 0) == ((lane & k) == 0)) ? min(v, u) : max(v, u);
        }
    return v;
}

// read ends per deep group (the groups' output offsets, scanned)
__global__ __launch_bounds__(256) void k_deep_count(const uint32_t* __restrict__ ndeep, const int32_t* __restrict__ dlist,
                                                    const int32_t* __restrict__ gend, const int32_t* __restrict__ rec_e,
                                                    uint32_t* __restrict__ gcnt) {
    __shared__ uint32_t s_w[4];
    const uint32_t nd = *ndeep;
    for (uint32_t gi = blockIdx.x; gi < nd; gi += gridDim.x) {
        const int64_t g0 = dlist[gi];
        const int32_t ge = gend[g0];
        const int64_t g1 = ge < 0 ? -1 - (int64_t)ge : (int64_t)ge;
        uint32_t c = 0;
        for (int64_t r = g0 + threadIdx.x; r < g1; r += 256) c += rec_e[r] >= 0 ? 1u : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o, 64);
        if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) gcnt[gi] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
        __syncthreads();
    }
}

struct DeepOut {   // the ranked slots k_fam_mark would have written
    int64_t R;
    uint32_t* rs_val;
    int32_t* mem_rec;
    uint8_t* segf;
    uint32_t* validf;
    uint4* mem_meta;
};

#ifdef DF_PROF   // phase timing of k_deep_fam (a measurement build: scripts/build_variant.sh NAME - -DDF_PROF)
__device__ unsigned long long g_df_prof[8];
#define DFP(k)                                                                      \
    do {                                                                            \
        __syncthreads();                                                            \
        if (t == 0) {                                                               \
            const unsigned long long now = wall_clock64();                          \
            atomicAdd(&g_df_prof[k], now - tp);                                     \
            tp = now;                                                               \
        }                                                                           \
    } while (0)
#else
#define DFP(k) __syncthreads()   // (each phase mark is a block barrier the kernel needs anyway)
#endif

__global__ __launch_bounds__(DF_T) void k_deep_fam(const uint32_t* __restrict__ ndeep, const int32_t* __restrict__ dlist,
                                                   const int32_t* __restrict__ gend, const int32_t* __restrict__ rec_e,
                                                   const uint64_t* __restrict__ rhash, const uint32_t* __restrict__ goff,
                                                   int64_t j0, PairView V, DevTable T, uint32_t* __restrict__ se,
                                                   int4* __restrict__ items, uint32_t* __restrict__ n_items,
                                                   int4* __restrict__ big, uint32_t* __restrict__ n_big,
                                                   uint32_t* __restrict__ ovf, uint32_t* __restrict__ err) {
    __shared__ unsigned long long s_key[DF_SLOTS];
    __shared__ int32_t s_rep[DF_SLOTS];
    __shared__ uint32_t s_cnt[DF_SLOTS];
    __shared__ uint16_t s_fid[DF_SLOTS];
    __shared__ int32_t s_list[DF_FAMS];
    __shared__ uint32_t s_base[DF_FAMS + 1];
    __shared__ uint32_t s_fill[DF_FAMS];
    __shared__ uint8_t s_wcnt[DF_T / 64][DF_FAMS];   // per wave and family: its ends in the sub-round
    __shared__ uint32_t s_w[DF_T / 64];
    __shared__ uint32_t s_nf, s_over;
    constexpr int U = 4;                       // records per thread per round (their loads in flight together)
    constexpr int U3 = 2;                      // (the placement round: registers)
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint64_t lt = (1ULL << lane) - 1ULL;
    const uint32_t nd = *ndeep;
    for (uint32_t gi = blockIdx.x; gi < nd; gi += gridDim.x) {
        const int64_t g0 = dlist[gi];
        const int32_t ge = gend[g0];
        const int64_t g1 = ge < 0 ? -1 - (int64_t)ge : (int64_t)ge;
#ifdef DF_PROF
        unsigned long long tp = wall_clock64();
#endif
        for (int i = t; i < DF_SLOTS; i += DF_T) {
            s_key[i] = DF_EMPTY;
            s_rep[i] = INT32_MAX;
            s_cnt[i] = 0u;
        }
        for (int i = t; i < (DF_T / 64) * DF_FAMS; i += DF_T) (&s_wcnt[0][0])[i] = 0;
        if (t == 0) { s_nf = 0u; s_over = 0u; }
        __syncthreads();
        // 1. the table: a slot per distinct tag hash, its lowest record and its end count
        for (int64_t c0 = g0; c0 < g1; c0 += (int64_t)U * DF_T) {
            int32_t ev[U];
            uint64_t hv[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int64_t r = c0 + k * DF_T + t;
                ev[k] = r < g1 ? rec_e[r] : -1;
            }
#pragma unroll
            for (int k = 0; k < U; ++k) hv[k] = ev[k] >= 0 ? rhash[c0 + k * DF_T + t] : 0ULL;
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const bool act = ev[k] >= 0;
                const uint64_t h = hv[k];
                const int32_t r = (int32_t)(c0 + k * DF_T + t);
                uint64_t todo = __ballot(act);
                while (todo) {
                    const int ld = __ffsll((long long)todo) - 1;   // the lowest lane: the lowest record
                    const uint64_t hl = shfl64(h, ld);
                    const uint64_t same = __ballot(act && h == hl) & todo;
                    if (lane == ld) {
                        uint32_t sl = df_slot0(hl);
                        int p = 0;
                        for (; p < DF_SLOTS; ++p) {
                            const unsigned long long prev = atomicCAS(&s_key[sl], DF_EMPTY, (unsigned long long)hl);
                            if (prev == DF_EMPTY || prev == hl) break;
                            sl = (sl + 1) & (DF_SLOTS - 1);
                        }
                        if (p == DF_SLOTS) s_over = 1u;
                        else {
                            atomicMin(&s_rep[sl], r);
                            atomicAdd(&s_cnt[sl], (uint32_t)__popcll(same));
                        }
                    }
                    todo &= ~same;
                }
            }
        }
        DFP(0);
        for (int i = t; i < DF_SLOTS; i += DF_T)
            if (s_key[i] != DF_EMPTY) {
                const uint32_t k = atomicAdd(&s_nf, 1u);
                if (k < (uint32_t)DF_FAMS) s_list[k] = i;
            }
        __syncthreads();
        const uint32_t nf = s_nf;
        if (nf > (uint32_t)DF_FAMS || s_over) {
            if (t == 0) atomicAdd(ovf, 1u);
            __syncthreads();
            continue;
        }
        // 2. family numbers in representative order (records are distinct), their offsets in the group,
        //    and the group's work items
        for (uint32_t i = t; i < nf; i += DF_T) {
            const int sl = s_list[i];
            const int32_t rep = s_rep[sl];
            uint32_t fid = 0;
            for (uint32_t k = 0; k < nf; ++k) fid += s_rep[s_list[k]] < rep ? 1u : 0u;
            s_fid[sl] = (uint16_t)fid;
            s_fill[fid] = 0u;
            s_base[fid] = s_cnt[sl];   // scanned below
        }
        __syncthreads();
        {
            const uint32_t c = t < (int)nf ? s_base[t] : 0u;   // nf <= DF_FAMS == DF_T
            uint32_t x = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
                if (lane >= o) x += y;
            }
            if (lane == 63) s_w[wv] = x;
            __syncthreads();
            uint32_t pre = x - c;
            for (int w = 0; w < wv; ++w) pre += s_w[w];
            if (t < (int)nf) {
                s_base[t] = pre;
                // families of up to 64 ends to k_deep_emit (a wave each), longer ones to k_deep_sortfam
                const int4 itm = make_int4((int32_t)(g0 + pre), (int32_t)c, (int32_t)(j0 + (int64_t)goff[gi] + pre), 0);
                if (c <= 64u) items[atomicAdd(n_items, 1u)] = itm;
                else big[atomicAdd(n_big, 1u)] = itm;
            }
            if (t == DF_T - 1) s_base[nf] = pre + c;
        }
        DFP(1);
        // 3. each end at its family's next slot in record order; every tag checked against its
        //    leader lane's, each leader's (after the round, all at once) against the representative's
        for (int64_t c0 = g0; c0 < g1; c0 += (int64_t)U3 * DF_T) {
            int32_t ev[U3];
            uint64_t hv[U3];
            int4 pt[U3];
#pragma unroll
            for (int k = 0; k < U3; ++k) {
                const int64_t r = c0 + k * DF_T + t;
                ev[k] = r < g1 ? rec_e[r] : -1;
            }
#pragma unroll
            for (int k = 0; k < U3; ++k) {
                hv[k] = ev[k] >= 0 ? rhash[c0 + k * DF_T + t] : 0ULL;
                pt[k] = ev[k] >= 0 ? V.tag[ev[k] >> 1] : make_int4(0, 0, 0, 0);
            }
            int32_t chk_rep[U3];
#pragma unroll
            for (int k = 0; k < U3; ++k) {
                const bool act = ev[k] >= 0;
                const uint64_t h = hv[k];
                const int32_t r = (int32_t)(c0 + k * DF_T + t);
                const TagKey mine = act ? tag_of_rec_np(T, r, pt[k]) : TagKey{};
                chk_rep[k] = -1;
                uint32_t myfid = 0, myrank = 0, lcnt = 0;
                uint64_t todo = __ballot(act);
                while (todo) {
                    const int ld = __ffsll((long long)todo) - 1;
                    const uint64_t hl = shfl64(h, ld);
                    const uint64_t same = __ballot(act && h == hl) & todo;
                    uint32_t fl = 0;
                    if (lane == ld) {
                        const int sl = df_find(s_key, hl);
                        if (sl < 0) atomicOr(err, EB_COLLISION);   // not reached (inserted in 1)
                        else {
                            fl = s_fid[sl];
                            lcnt = (uint32_t)__popcll(same);
                            s_wcnt[wv][fl] = (uint8_t)lcnt;
                            const int32_t rep = s_rep[sl];
                            if (rep != r) chk_rep[k] = rep;
                        }
                    }
                    fl = (uint32_t)__shfl((int)fl, ld, 64);
                    const TagKey lead = shfl_tag(mine, ld);
                    if ((same >> lane) & 1ULL) {
                        myfid = fl;
                        myrank = (uint32_t)__popcll(same & lt);
                        if (!tag_eq(mine, lead)) atomicOr(err, EB_COLLISION);
                    }
                    todo &= ~same;
                }
                __syncthreads();
                if (act) {
                    uint32_t o = s_base[myfid] + s_fill[myfid] + myrank;
                    for (int w = 0; w < wv; ++w) o += s_wcnt[w][myfid];
                    se[g0 + o] = (uint32_t)ev[k];
                }
                __syncthreads();
                if (lcnt) {
                    atomicAdd(&s_fill[myfid], lcnt);   // (lcnt: this lane led its family's lanes)
                    s_wcnt[wv][myfid] = 0;
                }
                __syncthreads();
            }
            // the leaders' representatives (loads of all of them in flight together)
            int32_t re[U3];
#pragma unroll
            for (int k = 0; k < U3; ++k) re[k] = chk_rep[k] >= 0 ? rec_e[chk_rep[k]] : 0;
#pragma unroll
            for (int k = 0; k < U3; ++k)
                if (chk_rep[k] >= 0) {
                    const int32_t r = (int32_t)(c0 + k * DF_T + t);
                    if (!tag_eq(tag_of_rec_np(T, r, pt[k]), tag_of_rec_np(T, chk_rep[k], V.tag[re[k] >> 1])))
                        atomicOr(err, EB_COLLISION);
                }
        }
        DFP(2);
    }
}

// One wave per family of up to 64 ends: the ranked slots, its ends sorted in the wave's registers
// when record order is not end order.
__device__ __forceinline__ void deep_put(const DeepOut& out, const PairView& V, const DevTable& T, int64_t j,
                                         uint32_t v, int32_t r, bool start, bool valid, uint32_t* err) {
    if (j >= out.R) { atomicOr(err, EB_PLAN); return; }   // not reached: the end counts are checked
    out.rs_val[j] = v;
    out.mem_rec[j] = r;
    out.segf[j] = start ? 1 : 0;
    out.validf[j] = valid ? 1u : 0u;
    if (out.mem_meta) out.mem_meta[j] = pack_meta(T, r, valid);
}

__global__ __launch_bounds__(256) void k_deep_emit(const int4* __restrict__ items, const uint32_t* __restrict__ n_items,
                                                   const uint32_t* __restrict__ se, PairView V, DevTable T, DeepOut out,
                                                   uint32_t* __restrict__ err) {
    const int lane = threadIdx.x & 63;
    const uint32_t ni = *n_items;
    const uint32_t nw = gridDim.x * (blockDim.x >> 6);
    for (uint32_t it = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); it < ni; it += nw) {
        const int4 d = items[it];
        const uint32_t m = (uint32_t)d.y;   // <= 64
        uint32_t v = lane < (int)m ? se[d.x + lane] : 0xffffffffu;
        const uint32_t nv = (uint32_t)__shfl_down((int)v, 1, 64);
        if (m > 1u && __any(lane + 1 < (int)m && nv < v)) v = wave_sort(v, lane);
        const uint32_t pv = (uint32_t)__shfl_up((int)v, 1, 64);
        if (lane < (int)m) {
            const int32_t r = (v & 1u) ? V.rec2[v >> 1] : V.rec1[v >> 1];
            deep_put(out, V, T, d.z + lane, v, r, lane == 0, lane == 0 || (v >> 1) != (pv >> 1), err);
        }
    }
}

// The families of more than 64 ends, one block each (a bitmap rank, below; else): runs of 64 sorted per wave, then
// merged pairwise in LDS, each value's place by a branch-free binary search in the other run (a
// thread's values searched in lockstep); the slots rewritten.
__global__ __launch_bounds__(DF_ST) void k_deep_sortfam(const int4* __restrict__ big, const uint32_t* __restrict__ n_big,
                                                        const uint32_t* __restrict__ se, PairView V, DevTable T,
                                                        DeepOut out, uint32_t* __restrict__ err) {
    __shared__ uint32_t s_a[DF_SORT], s_b[DF_SORT];   // (s_a: the bitmap of the rank path)
    __shared__ uint32_t s_w[DF_ST / 64], s_lo, s_hi;
    constexpr int SE = DF_SORT / DF_ST;
    constexpr uint32_t BM_WORDS = DF_SORT;            // rank path: ends within 32 * DF_SORT of each other
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t nu = *n_big;
    for (uint32_t q = blockIdx.x; q < nu; q += gridDim.x) {
        const int4 d = big[q];
        const uint32_t m = (uint32_t)d.y;
        if (m > (uint32_t)DF_SORT) {   // too long for the LDS sort: the pass re-runs on the sorted path
            if (t == 0) atomicOr(err, EB_DEEPSORT);
            continue;
        }
        // Rank path: a family's ends lie close together in end order (its pairs complete at one
        // position group), so a bitmap over [min, max] ranks them: an end's place is the number of
        // set bits before its own (the ends are distinct), and its pair's other end in the family
        // is the bit below an odd end ("line read twice").  No sort.
        uint32_t ev[SE];
        uint32_t lo = 0xffffffffu, hi = 0;
#pragma unroll
        for (int k = 0; k < SE; ++k) {
            const uint32_t i = (uint32_t)(k * DF_ST + t);
            ev[k] = i < m ? se[d.x + i] : 0xffffffffu;
            if (i < m) { lo = min(lo, ev[k]); hi = max(hi, ev[k]); }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, o, 64));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, o, 64));
        }
        __syncthreads();   // the last family's LDS use is done
        if (t == 0) { s_lo = 0xffffffffu; s_hi = 0u; }
        __syncthreads();
        if (lane == 0) { atomicMin(&s_lo, lo); atomicMax(&s_hi, hi); }
        __syncthreads();
        lo = s_lo;
        hi = s_hi;
        if (hi - lo < 32u * BM_WORDS) {
            const uint32_t nwd = ((hi - lo) >> 5) + 1;
            for (uint32_t x = t; x < nwd; x += DF_ST) s_a[x] = 0u;
            __syncthreads();
#pragma unroll
            for (int k = 0; k < SE; ++k) {
                const uint32_t i = (uint32_t)(k * DF_ST + t);
                if (i < m) atomicOr(&s_a[(ev[k] - lo) >> 5], 1u << ((ev[k] - lo) & 31));
            }
            __syncthreads();
            // exclusive prefix of the words' set bits: a contiguous run of words per thread
            const uint32_t per = (nwd + DF_ST - 1) / DF_ST;
            const uint32_t w0 = t * per, w1 = min(nwd, w0 + per);
            uint32_t run = 0;
            for (uint32_t x = w0; x < w1; ++x) run += (uint32_t)__popc(s_a[x]);
            uint32_t xs = run;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)xs, o, 64);
                if (lane >= o) xs += y;
            }
            if (lane == 63) s_w[wv] = xs;
            __syncthreads();
            uint32_t pre = xs - run;
            for (int w = 0; w < wv; ++w) pre += s_w[w];
            for (uint32_t x = w0; x < w1; ++x) {
                const uint32_t c = s_a[x];
                s_b[x] = pre;
                pre += (uint32_t)__popc(c);
            }
            __syncthreads();
            // each end's rank (registers), then the ends staged in LDS by rank (bit 31: the line read
            // twice) and the slots written in slot order: coalesced stores, the records gathered in end
            // order (scattered stores by rank cost partial-line write-backs)
            uint32_t rk[SE];
#pragma unroll
            for (int k = 0; k < SE; ++k) {
                const uint32_t i = (uint32_t)(k * DF_ST + t);
                rk[k] = 0xffffffffu;
                if (i >= m) continue;
                const uint32_t v = ev[k], b = v - lo, wd = b >> 5, bit = b & 31;
                rk[k] = s_b[wd] + (uint32_t)__popc(s_a[wd] & ((1u << bit) - 1u));
                // the pair's first end (v - 1) in the family: this second end is its line read twice
                const bool twice = (v & 1u) && b > 0 && ((s_a[(b - 1) >> 5] >> ((b - 1) & 31)) & 1u);
                ev[k] = v | (twice ? 0x80000000u : 0u);
            }
            __syncthreads();   // the bitmap and the word prefixes are read
#pragma unroll
            for (int k = 0; k < SE; ++k)
                if (rk[k] != 0xffffffffu) s_a[rk[k]] = ev[k];
            __syncthreads();
            if ((int64_t)d.z + (int64_t)m > out.R) {   // not reached: the end counts are checked
                if (t == 0) atomicOr(err, EB_PLAN);
                continue;
            }
            for (uint32_t j0 = 0; j0 < m; j0 += 4u * DF_ST) {
                uint32_t a[4];
                int32_t r[4];
                uint4 mt[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t j = j0 + (uint32_t)(u * DF_ST + t);
                    a[u] = j < m ? s_a[j] : 0u;
                    const uint32_t v = a[u] & 0x7fffffffu;
                    r[u] = j < m ? ((v & 1u) ? V.rec2[v >> 1] : V.rec1[v >> 1]) : 0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t j = j0 + (uint32_t)(u * DF_ST + t);
                    mt[u] = j < m && out.mem_meta ? T.meta[CC_IDX(r[u], T.n, DS_MEMBER)] : make_uint4(0u, 0u, 0u, 0u);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t j = j0 + (uint32_t)(u * DF_ST + t);
                    if (j >= m) continue;
                    const int64_t o = (int64_t)d.z + j;
                    const bool valid = !(a[u] >> 31);
                    out.rs_val[o] = a[u] & 0x7fffffffu;
                    out.mem_rec[o] = r[u];
                    out.segf[o] = j == 0 ? 1 : 0;
                    out.validf[o] = valid ? 1u : 0u;
                    if (out.mem_meta) {
                        uint4 x = mt[u];
                        x.w |= (valid ? 1u : 0u) << 23;
                        out.mem_meta[o] = x;
                    }
                }
            }
            continue;
        }
        uint32_t p2 = 128;
        while (p2 < m) p2 <<= 1;
        __syncthreads();
        {
            uint32_t v[SE];
#pragma unroll
            for (int k = 0; k < SE; ++k) {
                const uint32_t i = (uint32_t)(k * DF_ST + t);
                v[k] = i < m ? se[d.x + i] : 0xffffffffu;
            }
#pragma unroll
            for (int k = 0; k < SE; ++k) {
                const uint32_t i = (uint32_t)(k * DF_ST + t);
                if (k * DF_ST >= (int)p2) break;              // (uniform over the block)
                s_a[i] = wave_sort(v[k], lane);               // 64-aligned runs: one wave's values
            }
        }
        __syncthreads();
        uint32_t* A = s_a;
        uint32_t* B = s_b;
        for (uint32_t w = 64; w < p2; w <<= 1) {
            for (int h = 0; h < SE; h += SE / 2) {   // (in halves: registers)
                uint32_t v[SE / 2], lo[SE / 2];
#pragma unroll
                for (int k = 0; k < SE / 2; ++k) {
                    const uint32_t i = (uint32_t)((h + k) * DF_ST + t);
                    v[k] = i < p2 ? A[i] : 0u;
                    lo[k] = (i & ~(2 * w - 1)) + ((i & w) ? 0u : w);
                }
                // lo: the position in the other run, from its start; the first run's values count the
                // other's smaller ones, the second's also the equal ones (the padding): a stable merge
                for (uint32_t sp = w >> 1; sp > 0; sp >>= 1) {
#pragma unroll
                    for (int k = 0; k < SE / 2; ++k) {
                        const uint32_t i = (uint32_t)((h + k) * DF_ST + t);
                        const uint32_t pm = A[lo[k] + sp - 1];
                        if ((i & w) ? (pm <= v[k]) : (pm < v[k])) lo[k] += sp;
                    }
                }
#pragma unroll
                for (int k = 0; k < SE / 2; ++k) {
                    const uint32_t i = (uint32_t)((h + k) * DF_ST + t);
                    if (i >= p2) continue;
                    const uint32_t pm = A[lo[k]];
                    if ((i & w) ? (pm <= v[k]) : (pm < v[k])) lo[k] += 1;
                    const uint32_t st = i & ~(2 * w - 1), other = st + ((i & w) ? 0u : w);
                    B[st + (i & (w - 1)) + (lo[k] - other)] = v[k];
                }
            }
            __syncthreads();
            uint32_t* tmp = A; A = B; B = tmp;
        }
        // the slots, the records of a thread's ends gathered together (in halves: registers)
        for (int h = 0; h < SE; h += SE / 2) {
            uint32_t v[SE / 2];
            int32_t r[SE / 2];
#pragma unroll
            for (int k = 0; k < SE / 2; ++k) {
                const uint32_t i = (uint32_t)((h + k) * DF_ST + t);
                v[k] = i < m ? A[i] : 0u;
                r[k] = i < m ? ((v[k] & 1u) ? V.rec2[v[k] >> 1] : V.rec1[v[k] >> 1]) : 0;
            }
#pragma unroll
            for (int k = 0; k < SE / 2; ++k) {
                const uint32_t i = (uint32_t)((h + k) * DF_ST + t);
                if (i < m) deep_put(out, V, T, d.z + (int64_t)i, v[k], r[k], i == 0, i == 0 || (v[k] >> 1) != (A[i - 1] >> 1), err);
            }
        }
    }
}

// family starts, and per family the members dropped as the second end of a pair already in it
// (rare; fam_drop zeroed beforehand)
__global__ __launch_bounds__(256) void k_fam_build(int64_t F, int64_t R, const int32_t* __restrict__ fam_beg,
                                                   const int32_t* __restrict__ fam_drop,
                                                   const uint32_t* __restrict__ rs_val, const uint64_t* __restrict__ rs_key,
                                                   const int32_t* __restrict__ pr_region, const uint64_t* __restrict__ rhash,
                                                   const int32_t* __restrict__ mem_rec, int32_t* __restrict__ fam_end,
                                                   int32_t* __restrict__ fam_n, int32_t* __restrict__ fam_first,
                                                   int32_t* __restrict__ fam_region, uint64_t* __restrict__ fam_hash,
                                                   uint8_t* __restrict__ cflag, int32_t* __restrict__ cfam,
                                                   int32_t* __restrict__ fam_o, PairView V, DevTable T,
                                                   TagKey* __restrict__ fam_tag, int32_t* __restrict__ fam_rec) {
    int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f < F) {
        fam_o[f] = 0x7f7f7f7f;   // orphan tags are never processed (k_entries_build sets the others)
        int32_t b = fam_beg[f];
        int32_t e = (f + 1 < F) ? fam_beg[f + 1] : (int32_t)R;
        fam_end[f] = e;
        fam_n[f] = e - b - fam_drop[f];   // len(read_dict[tag]): members not dropped
        uint32_t fe = rs_val[b];
        fam_first[f] = (int32_t)fe;
        fam_region[f] = pr_region[fe >> 1];
        fam_hash[f] = rhash ? rhash[mem_rec[b]] : rs_key[b];   // the full tag hash (deep keys are truncated)
        cflag[fe] = 1;
        cfam[fe] = (int32_t)f;
        // the family's tag for the DCS / SC joins, in the passes whose stage joins (k_fam_tags' value)
        // and its first member's record (the joins' t_rec / p_rec)
        if (fam_tag) {
            const int32_t r0 = mem_rec[b];
            fam_tag[f] = tag_of_rec(T, r0, V.tag[fe >> 1]);
            fam_rec[f] = r0;
        }
    }
}

// per family its tag, for the DCS / SC joins (built when a stage joins the grouping, ensure_fam_tags)
__global__ __launch_bounds__(256) void k_fam_tags(int64_t F, const int32_t* __restrict__ fam_first,
                                                  const int32_t* __restrict__ fam_beg, const int32_t* __restrict__ mem_rec,
                                                  PairView V, DevTable T, TagKey* __restrict__ fam_tag,
                                                  int32_t* __restrict__ fam_rec) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f < F) {
        const int32_t r0 = mem_rec[fam_beg[f]];
        fam_tag[f] = tag_of_rec(T, r0, V.tag[fam_first[f] >> 1]);
        fam_rec[f] = r0;
    }
}

__global__ __launch_bounds__(256) void k_csn_keys(int64_t F, const int32_t* __restrict__ fam_by_k,
                                                  const int32_t* __restrict__ fam_first, const uint64_t* __restrict__ chash,
                                                  uint64_t* __restrict__ ekey, uint32_t* __restrict__ eval) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= F) return;
    int32_t f = fam_by_k[k];
    ekey[k] = chash[fam_first[f] >> 1];
    eval[k] = (uint32_t)k;
}

__global__ __launch_bounds__(256) void k_csn_mark(int64_t F, const uint64_t* __restrict__ es_key,
                                                  const uint32_t* __restrict__ es_val, const int32_t* __restrict__ fam_by_k,
                                                  const int32_t* __restrict__ fam_first, PairView V, DevTable T,
                                                  uint32_t* __restrict__ segf, uint32_t* __restrict__ err) {
    int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= F) return;
    bool start = (j == 0) || es_key[j - 1] != es_key[j];
    if (!start) {
        int32_t pa = fam_first[fam_by_k[es_val[j]]] >> 1, pb = fam_first[fam_by_k[es_val[j - 1]]] >> 1;
        if (!ckey_eq(ckey_of_pair(T, V, pa), ckey_of_pair(T, V, pb))) {
            atomicOr(err, EB_COLLISION);
            start = true;
        }
    }
    segf[j] = start;
}

// Overlapping bed regions (a record streamed by two regions): the reference's region loop emits an
// entry with both tags at the end of the region that completed it and deletes its families from
// read_dict (SSCS_maker.py:312-339); a pair completing one of those families again in a later region
// (the same reads fetched by the overlapping region) then reads read_dict[tag] -> KeyError
// (consensus_helper.py:490).  One thread per entry: any member pair completed in a region after the
// entry's completing region raises it.
__global__ __launch_bounds__(256) void k_overlap_keyerror(int64_t E, const int32_t* __restrict__ ent_f,
                                                          const int32_t* __restrict__ fam_beg,
                                                          const int32_t* __restrict__ fam_end,
                                                          const int32_t* __restrict__ fam_region,
                                                          const uint32_t* __restrict__ rs_val,
                                                          const int32_t* __restrict__ pr_region,
                                                          uint32_t* __restrict__ err) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= E) return;
    const int32_t fa = ent_f[2 * q], fb = ent_f[2 * q + 1];
    if (fb < 0) return;   // an entry with one tag is never emitted, its families never deleted
    const int32_t rc = max(fam_region[fa], fam_region[fb]);
    bool late = false;
    for (int k = 0; k < 2 && !late; ++k) {
        const int32_t f = k ? fb : fa;
        for (int32_t j = fam_beg[f]; j < fam_end[f] && !late; ++j) late = pr_region[rs_val[j] >> 1] > rc;
    }
    if (late) atomicOr(err, EB_KEYERROR);
}

// one thread per csn segment: first two creation events form the csn_pair_dict entry
// (consensus_helper.py:470-489); later ones are "NOT UNIQUE" orphans.
__global__ __launch_bounds__(256) void k_csn_entries(int64_t F, const uint32_t* __restrict__ segf,
                                                     const uint32_t* __restrict__ es_val,
                                                     const int32_t* __restrict__ fam_by_k,
                                                     const int32_t* __restrict__ fam_region,
                                                     uint8_t* __restrict__ emark, int32_t* __restrict__ e1k,
                                                     uint32_t* __restrict__ err, unsigned long long* __restrict__ cnt) {
    int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= F || !segf[j]) return;
    int64_t m = 1;
    while (j + m < F && !segf[j + m]) ++m;
    uint32_t k0 = es_val[j];
    int32_t reg0 = fam_region[fam_by_k[k0]];
    for (int64_t i = 1; i < m; ++i)
        if (fam_region[fam_by_k[es_val[j + i]]] != reg0) atomicOr(err, EB_AMBIGUOUS);
    if (m > 2) atomicAdd(&cnt_stripe(cnt)[CC_CNT_ORPHAN_TAGS], (unsigned long long)(m - 2));
    emark[k0] = 1;
    e1k[k0] = m > 1 ? (int32_t)es_val[j + 1] : -1;
}

// csn_pair_dict fast path.  Creation events (new tags) of one pair are consecutive in creation
// order and share the pair's consensus tag; unless a consensus tag is shared by families created by
// different pairs ("Consensus tag NOT UNIQUE" territory, consensus_helper.py:470-489), every entry
// is exactly one creating pair's events.  Sharing is detected over the creating pairs' consensus
// key hashes (equal hashes count as shared: the exact sort path then decides).  Two pairs with one
// consensus key have their ends at the same two positions.  When the stream is the coordinate-
// sorted table itself (ident), both complete in the position group of the later end, so with both
// ends in small groups (at most GRP_SMALL records, so at most GRP_SMALL completing pairs of up to
// two creation events each) their start entries are less than CW apart: those are checked in LDS
// per tile of CT entries plus the CW before it; the others (an end in a deep group, or another
// stream) in a global hash table.  Both pairs of a shared key classify alike (same positions, so
// same groups).
// CT entries per tile and a table of CSLOTS >= CT + CW + 1 slots (every start of the tile and its
// window fits): 20.6 KB of LDS per block, 7 blocks per CU
constexpr int64_t CT = 1024;
constexpr int CW = 2 * GRP_SMALL;   // start entries of one small group's pairs are < CW apart
constexpr int CSLOTS = 2048;
static_assert(CSLOTS >= CT + CW + 1, "the tile table holds every start of the tile and its window");
__global__ __launch_bounds__(256) void k_csn_fast(int64_t F, const int32_t* __restrict__ pair_by_k,
                                                  const uint64_t* __restrict__ chash,
                                                  const uint32_t* __restrict__ bigE,
                                                  unsigned long long* __restrict__ ht_key, uint64_t mask,
                                                  uint8_t* __restrict__ emark, int32_t* __restrict__ e1k,
                                                  uint32_t* __restrict__ shared) {
    __shared__ int32_t s_p[CT + CW + 2];
    __shared__ unsigned long long s_tab[CSLOTS];
    const int t = threadIdx.x;
    const int64_t t0 = (int64_t)blockIdx.x * CT, t1 = min(F, t0 + CT);
    const int64_t w0 = max((int64_t)0, t0 - CW - 1), w1 = min(F, t1 + 1);
    for (int64_t k = w0 + t; k < w1; k += blockDim.x) s_p[k - w0] = pair_by_k[k];
    for (int i = t; i < CSLOTS; i += blockDim.x) s_tab[i] = ~0ULL;
    __syncthreads();
    bool sh = false;
    for (int64_t k = (w0 == 0 ? 0 : w0 + 1) + t; k < t1; k += blockDim.x) {
        const int32_t p = s_p[k - w0];
        const bool start = (k == 0) || s_p[k - 1 - w0] != p;
        if (k >= t0) {
            emark[k] = start ? 1 : 0;
            if (start) e1k[k] = (k + 1 < F && s_p[k + 1 - w0] == p) ? (int32_t)(k + 1) : -1;
        }
        if (!start) continue;
        const unsigned long long h = chash[p];
        if (bigE && !bigE[2 * p] && !bigE[2 * p + 1]) {
            // both ends in small groups: the tile's table
            uint32_t slot = (uint32_t)(h >> 13) & (CSLOTS - 1);
            bool done = false;
            for (int i = 0; i < CSLOTS && !done; ++i) {
                const unsigned long long prev = atomicCAS(&s_tab[slot], ~0ULL, h);
                if (prev == ~0ULL) done = true;
                else if (prev == h) { sh = true; done = true; }
                else slot = (slot + 1) & (CSLOTS - 1);
            }
            if (!done) sh = true;
        } else if (k >= t0) {
            uint64_t slot = h & mask;
            bool done = false;
            for (uint64_t i = 0; i <= mask && !done; ++i) {
                const unsigned long long prev = atomicCAS(&ht_key[slot], ~0ULL, h);
                if (prev == ~0ULL) done = true;
                else if (prev == h) { sh = true; done = true; }
                else slot = (slot + 1) & mask;
            }
            if (!done) sh = true;   // table full: the exact sort path decides
        }
    }
    if (sh) *shared = 1u;
}

// ------------------------------------------------------------------ SSCS emission + vote

// One thread per csn_pair_dict entry with two tags: its two emitted families (SSCS_maker.py:312-339)
// and, once per entry, the sscs_qname fields both records are named after (consensus_helper.py:
// 199-249; the host formats the names).
__global__ __launch_bounds__(256) void k_sscs_emit(int64_t E, const int32_t* __restrict__ ent_f,
                                                   const int32_t* __restrict__ ent_pair,
                                                   const uint8_t* __restrict__ has2, const uint32_t* __restrict__ hx,
                                                   const int32_t* __restrict__ fam_n, const int32_t* __restrict__ fam_beg,
                                                   const int32_t* __restrict__ fam_end,
                                                   const int32_t* __restrict__ mem_rec, int32_t* __restrict__ emit_fam,
                                                   int32_t* __restrict__ emit_n, int32_t* __restrict__ emit_rec,
                                                   uint8_t* __restrict__ needv, int2* __restrict__ emit_span,
                                                   PairView V, DevTable T, int32_t* __restrict__ ent_ckey) {
    int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= E || !has2[r]) return;
    const uint32_t x = hx[r];
    const uint32_t o = 2 * x;
    // every load of the entry first (both families, then their first members, and the pair's
    // consensus key), the stores after
    const int2 ff = *reinterpret_cast<const int2*>(ent_f + 2 * r);
    const int32_t f2[2] = {ff.x, ff.y};
    int32_t b2[2], n2[2], e2[2], m2[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) { b2[s] = fam_beg[f2[s]]; n2[s] = fam_n[f2[s]]; e2[s] = fam_end[f2[s]]; }
#pragma unroll
    for (int s = 0; s < 2; ++s) m2[s] = mem_rec[b2[s]];
    const CKey c = ckey_of_pair(T, V, ent_pair[r]);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        emit_fam[o + s] = f2[s];
        emit_n[o + s] = n2[s];
        emit_rec[o + s] = m2[s];
        needv[o + s] = n2[s] >= 2 ? 1 : 0;
        emit_span[o + s] = make_int2(b2[s], e2[s] - b2[s]);   // the vote plan's member range, by emit slot
    }
    int32_t* out = ent_ckey + 9 * (int64_t)x;
    out[0] = c.bc; out[1] = c.tidLo; out[2] = c.posLo; out[3] = c.tidHi; out[4] = c.posHi;
    out[5] = c.cigA; out[6] = c.cigB; out[7] = (int32_t)(c.strand & 3u); out[8] = (int32_t)c.abstlen;
}


// Mode of a per-member value over the valid members of [beg,end) in member order:
// Counter(...).most_common() with first-seen tie break (randint -> 0), and for
// flags the 99 > 83 > 147 > 163 priority of consensus_flag (consensus_helper.py:509-565).
template <typename Get>
__device__ int32_t wave_mode(int lane, int32_t beg, int32_t end, const int32_t* __restrict__ mem_rec,
                             const uint32_t* __restrict__ mem_valid, Get get, bool is_flag) {
    int32_t v0 = get(mem_rec[beg]);
    bool diff = false;
    for (int32_t jb = beg; jb < end; jb += 64) {
        int32_t j = jb + lane;
        bool d = (j < end) && mem_valid[j] && get(mem_rec[j]) != v0;
        if (__any(d)) { diff = true; break; }
    }
    if (!diff) return v0;
    // slow path: per candidate (first occurrence) count; best = max count, ties -> earliest
    int32_t best_cnt = -1, best_idx = INT_MAX, best_val = v0;
    bool has99 = false, has83 = false, has147 = false, has163 = false;
    // pass 1: the maximum count
    for (int32_t jb = beg; jb < end; jb += 64) {
        int32_t j = jb + lane;
        bool mine = (j < end) && mem_valid[j];
        int32_t v = mine ? get(mem_rec[j]) : 0;
        int32_t c = 0;
        bool first = mine;
        for (int32_t k = beg; k < end; ++k) {
            if (!mem_valid[k]) continue;
            int32_t w = get(mem_rec[k]);
            if (mine && w == v) {
                ++c;
                if (k < j) first = false;
            }
        }
        if (first) {
            if (c > best_cnt || (c == best_cnt && j < best_idx)) { best_cnt = c; best_idx = j; best_val = v; }
        }
    }
    // wave reduce (max count, min index)
    for (int o = 32; o > 0; o >>= 1) {
        int32_t oc = __shfl_xor(best_cnt, o), oi = __shfl_xor(best_idx, o), ov = __shfl_xor(best_val, o);
        if (oc > best_cnt || (oc == best_cnt && oi < best_idx)) { best_cnt = oc; best_idx = oi; best_val = ov; }
    }
    if (!is_flag) return best_val;
    // consensus_flag: if several flags share the max count, prefer 99, 83, 147, 163
    for (int32_t jb = beg; jb < end; jb += 64) {
        int32_t j = jb + lane;
        bool mine = (j < end) && mem_valid[j];
        int32_t v = mine ? get(mem_rec[j]) : 0;
        int32_t c = 0;
        if (mine && (v == 99 || v == 83 || v == 147 || v == 163)) {
            for (int32_t k = beg; k < end; ++k)
                if (mem_valid[k] && get(mem_rec[k]) == v) ++c;
        }
        bool hit = mine && c == best_cnt;
        has99 |= __any(hit && v == 99);
        has83 |= __any(hit && v == 83);
        has147 |= __any(hit && v == 147);
        has163 |= __any(hit && v == 163);
    }
    int nties = 0;  // are there several values at the max count?
    for (int32_t jb = beg; jb < end; jb += 64) {
        int32_t j = jb + lane;
        bool mine = (j < end) && mem_valid[j];
        int32_t v = mine ? get(mem_rec[j]) : 0;
        bool first = mine;
        int32_t c = 0;
        if (mine) {
            for (int32_t k = beg; k < end; ++k) {
                if (!mem_valid[k]) continue;
                if (get(mem_rec[k]) == v) { ++c; if (k < j) first = false; }
            }
        }
        nties += __popcll(__ballot(first && c == best_cnt));
    }
    if (nties == 1) return best_val;
    if (has99) return 99;
    if (has83) return 83;
    if (has147) return 147;
    if (has163) return 163;
    return best_val;
}

// ---- families above VOTE_BIGN members: the members split over waves ------------------------
// consensus_maker (SSCS_maker.py:81-168) for families of any size, in two kernels.  k_big_swar: the
// family's members in chunks of BIG_CH (= VOTE_BIGN, so byte counters cannot overflow) are work
// items voted exactly like k_sscs_vote_swar's families (lane = 16 positions, byte-sliced counts),
// each item writing its per-position pass / A / C / G counts as four byte planes.  k_big_final: one
// wave per family sums its items' planes (lane = 4 positions), applies the exact cutoff and the
// quality rule (60 when count[best] >= 2, every passing quality being >= 30; the one passing
// member's quality when count[best] == 1; 0 when nothing passes), checks every member once (short
// read, qualities, cigar, RG) and takes the create_aligned_segment modes (consensus_helper.py:
// 509-565) with an LDS hash table: count and first occurrence per distinct value, then the first
// maximum (randint -> 0) and the flag priority 99 > 83 > 147 > 163.  A family of n members costs
// n / BIG_CH item-lanes side by side and its modes O(n), not O(n^2).
constexpr int BIG_CH = 63;    // members per item (VOTE_BIGN)
constexpr int BIG_STAGE = 6;  // items per wave whose member records k_big_swar stages in LDS
constexpr int BIG_PL = 4;     // byte planes per item: pass, A, C x 2, G x 4 counts

// Counters of members [jb0, jend) at positions i0..i0+3 (< L) of one lane; any base code.
__device__ __forceinline__ void big_count(int32_t jb0, int32_t jend, int32_t L, int32_t i0, int lane,
                                          const uint4* __restrict__ mem_meta, const DevTable& T, uint32_t (&cnt)[4][4],
                                          uint32_t (&qs)[4][4], uint32_t (&fail)[4], uint32_t& eb) {
    const bool act = i0 < L;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        fail[t] = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) { cnt[t][b] = 0; qs[t][b] = 0; }
    }
    for (int32_t jb = jb0; jb < jend; jb += 64) {
        const int32_t j = jb + lane;
        uint4 m = make_uint4(0, 0, 0, 0);
        if (j < jend) m = mem_meta[j];
        const bool v = (m.w >> 23) & 1u;
        const uint32_t ls = m.z & 0xffffu;
        const uint64_t my_q = (uint64_t)m.x << 4;
        const uint64_t my_s = my_q + (uint64_t)((ls + 15u) & ~15u);
        const int32_t my_ls = v ? (int32_t)ls : 0;   // positions of this member (0: skip it)
        const int cm = min(64, jend - jb);
        for (int k0 = 0; k0 < cm; k0 += 4) {
            uint32_t q4v[4], s2v[4];
            int32_t lsv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + u < cm ? k0 + u : 0;
                lsv[u] = k0 + u < cm ? readlane_i32(my_ls, k) : 0;
                q4v[u] = 0;
                s2v[u] = 0;
                if (act && i0 < lsv[u]) {
                    const uint64_t qo = readlane_u64(my_q, k), so = readlane_u64(my_s, k);
                    q4v[u] = *reinterpret_cast<const uint32_t*>(T.payload + qo + i0);
                    s2v[u] = *reinterpret_cast<const uint16_t*>(T.payload + so + (i0 >> 1));
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t q4 = q4v[u], s2 = s2v[u];
                const uint32_t nib[4] = {(s2 >> 4) & 15u, s2 & 15u, (s2 >> 12) & 15u, (s2 >> 8) & 15u};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (i0 + t >= L || i0 + t >= lsv[u]) break;
                    const uint32_t q = (q4 >> (8 * t)) & 0xffu;
                    const uint32_t b = nib[t];
                    if (!(b == 1u || b == 2u || b == 4u || b == 8u || b == 15u)) eb |= EB_BAD_BASE;
                    if (q < 30u) fail[t] += 1;
                    else {
                        if (b == 15u) eb |= EB_N_HIGHQ;
#pragma unroll
                        for (int bb = 0; bb < 4; ++bb)
                            if (b == (1u << bb)) { cnt[t][bb] += 1; qs[t][bb] += q; }
                    }
                }
            }
        }
    }
}

// consensus length of a large family: member 0's query length, 0 without a cigar or beyond the
// table's longest read (the final kernel reports both)
__device__ __forceinline__ int32_t big_len(const uint4& m0, int32_t max_len) {
    const uint32_t ql0 = m0.z >> 16;
    const int32_t L = ql0 == 0xffffu ? 0 : (int32_t)ql0;
    return L > max_len ? 0 : L;
}

// Mode of a per-member value over the valid members of [beg, end) with an LDS hash table (one wave,
// the block's only one): per distinct value its count and first member; the first maximum wins
// (Counter.most_common order with randint -> 0), flags take 99 > 83 > 147 > 163 among the maxima.
// *overflow when the values do not fit the table (the caller falls back to wave_mode).
constexpr int MODE_SLOTS = 256;
constexpr int32_t MODE_EMPTY = INT_MIN;
template <typename Get>
__device__ int32_t lds_mode(int lane, int32_t beg, int32_t end, const uint4* __restrict__ meta, Get get, bool is_flag,
                            int32_t* s_key, uint32_t* s_cnt, uint32_t* s_first, bool* overflow) {
    for (int i = lane; i < MODE_SLOTS; i += 64) { s_key[i] = MODE_EMPTY; s_cnt[i] = 0; s_first[i] = 0xffffffffu; }
    __syncthreads();
    bool ovf = false;
    for (int32_t jb = beg; jb < end; jb += 64) {
        const int32_t j = jb + lane;
        const bool in = j < end && ((meta[j].w >> 23) & 1u);
        const int32_t val = in ? get(j) : 0;
        if (in && val == MODE_EMPTY) ovf = true;
        // the lanes holding one value are served by their lowest lane (its member is their first):
        // one set of LDS atomics per distinct value, not one per member (most members carry the
        // family's common value, and same-word LDS atomics serialise)
        uint64_t todo = __ballot(in && val != MODE_EMPTY);
        while (todo) {
            const int ld = __ffsll((long long)todo) - 1;
            const int32_t vl = __shfl(val, ld, 64);
            const uint64_t same = __ballot(in && val == vl) & todo;
            if (lane == ld) {
                uint32_t h = ((uint32_t)vl * 0x9E3779B1u) >> 24;   // 8 bits: MODE_SLOTS == 256
                bool done = false;
                for (int pr = 0; pr < MODE_SLOTS && !done; ++pr) {
                    const int32_t prev = atomicCAS(&s_key[h], MODE_EMPTY, vl);
                    if (prev == MODE_EMPTY || prev == vl) {
                        atomicAdd(&s_cnt[h], (uint32_t)__popcll(same));
                        atomicMin(&s_first[h], (uint32_t)(j - beg));
                        done = true;
                    } else {
                        h = (h + 1) & (MODE_SLOTS - 1);
                    }
                }
                if (!done) ovf = true;
            }
            todo &= ~same;
        }
        __syncthreads();
    }
    *overflow = __any(ovf);
    // first maximum: (count desc, first asc) over the slots, four per lane
    uint32_t bc = 0, bf = 0xffffffffu;
    int32_t bv = 0;
    for (int i = lane; i < MODE_SLOTS; i += 64) {
        const uint32_t c = s_cnt[i], f = s_first[i];
        if (c > bc || (c == bc && c > 0 && f < bf)) { bc = c; bf = f; bv = s_key[i]; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t oc = __shfl_xor(bc, o), of = __shfl_xor(bf, o);
        const int32_t ov = __shfl_xor(bv, o);
        if (oc > bc || (oc == bc && of < bf)) { bc = oc; bf = of; bv = ov; }
    }
    if (is_flag) {
        // several values at the maximum: the proper-pair priority (consensus_flag)
        int nmax = 0;
        bool h99 = false, h83 = false, h147 = false, h163 = false;
        for (int i = lane; i < MODE_SLOTS; i += 64) {
            if (s_cnt[i] != bc || bc == 0) continue;
            ++nmax;
            const int32_t v = s_key[i];
            h99 |= v == 99; h83 |= v == 83; h147 |= v == 147; h163 |= v == 163;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) nmax += __shfl_xor(nmax, o);
        h99 = __any(h99); h83 = __any(h83); h147 = __any(h147); h163 = __any(h163);
        if (nmax > 1) {
            if (h99) bv = 99;
            else if (h83) bv = 83;
            else if (h147) bv = 147;
            else if (h163) bv = 163;
        }
    }
    __syncthreads();
    return bv;
}

// Work items of the large families (k_vote_plan listed them): a family of two or more chunks gets
// consecutive items, big_item[k] its first (-1: one chunk, counted by k_big_final itself).  The
// item count was planned: beyond the capacity the pass re-runs exactly (EB_PLAN).
__global__ __launch_bounds__(256) void k_big_items(const uint32_t* __restrict__ d_nbig, const int32_t* __restrict__ slow_list,
                                                   const int32_t* __restrict__ vote_fam,
                                                   const int32_t* __restrict__ fam_beg, const int32_t* __restrict__ fam_end,
                                                   int64_t cap, uint32_t* __restrict__ d_items, int32_t* __restrict__ big_item,
                                                   int4* __restrict__ items, uint32_t* __restrict__ err) {
    const int64_t nb = (int64_t)*d_nbig;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nb; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = slow_list[k];
        const int32_t f = vote_fam[v];
        const int32_t beg = fam_beg[f], cnt = fam_end[f] - beg;
        const int32_t nch = (cnt + BIG_CH - 1) / BIG_CH;
        if (nch <= 1) { big_item[k] = -1; continue; }
        const uint32_t base = atomicAdd(d_items, (uint32_t)nch);
        big_item[k] = (int32_t)base;
        if ((int64_t)base + nch > cap) { atomicOr(err, EB_PLAN); continue; }
        for (int32_t c = 0; c < nch; ++c)
            items[base + c] = make_int4(v, beg, beg + c * BIG_CH, min(BIG_CH, cnt - c * BIG_CH));
    }
}

// ---- SWAR vote for families of at most VOTE_BIGN members ----------------------------------
// consensus_maker (SSCS_maker.py:81-168) as byte-sliced integer work.  One lane owns one
// 16-position chunk of one family.  Per member it makes one 16-B load of qualities and one 8-B
// load of BAM nibbles, then updates four 32-bit words of four positions each (the even and the
// odd positions of each 8-position half, so a nibble word unpacks with one shift and mask):
//   pc   members with q >= 30 at the position ("phred pass")
//   ca   passing A, cc passing C (x2), cg passing G (x4)        (T = pc - A - C - G)
//   orb  OR of the passing base codes (one-hot: ACGT = 1,2,4,8)
//   ql   quality of the last passing member
// about 15 integer instructions per word per member.  A passing N (code 15, the IndexError of
// SSCS_maker.py:129) makes orb non-one-hot, so its position takes the per-position path, which
// re-reads the position when orb is 15 (passing_n).
// The molecular quality needs no per-base quality sums (Q4): every passing quality is >= 30, so
// min(60, sum of the best base's qualities) is 60 once count[best] >= 2, min(60, q) of the lone
// passing member when count[best] == 1 == pass, and 0 when count[best] == 0.  Positions where the
// passing members agree (orb one-hot) resolve in SWAR; the rest resolve per position from the byte
// counters (first maximum in A,C,G,T order, the exact cutoff through thr[]), and the rare
// count[best] == 1 < pass re-reads that one position.  Families with more than VOTE_BIGN members
// go to the split vote (k_big_partial / k_big_final) through a device-counted hand-over list.
constexpr int VOTE_BIGN = 63;   // byte counters: cg holds 4 x count <= 252
constexpr int SV_POS = 16;      // positions per lane
#ifndef CC_SV_U
#define CC_SV_U 2
#endif
#ifndef CC_SV_WAVES
#define CC_SV_WAVES 1
#endif
constexpr int SV_U = CC_SV_U;   // members whose loads are in flight together
#ifndef CC_BIG_U
#define CC_BIG_U CC_SV_U
#endif
constexpr int BIG_U = CC_BIG_U;  // the same for the large families' items (k_big_swar)

// thr[p] = min{c : (double)c / p >= cutoff} for p = 1..VOTE_BIGN (p + 1 when none): the exact
// Python comparison of SSCS_maker.py:154-155 turned into an integer test, once per launch.
__global__ void k_cutoff_table(double cutoff, int32_t* __restrict__ thr) {
    const int p = threadIdx.x;
    if (p > VOTE_BIGN) return;
    int32_t t = p + 1;
    if (p > 0)
        for (int c = 0; c <= p; ++c)
            if ((double)c / (double)p >= cutoff) { t = c; break; }
    thr[p] = t;
}

// Exact mode of one family by a single thread (mixed families only): Counter.most_common with the
// first-seen tie break (randint -> 0); for flags the 99 > 83 > 147 > 163 priority of
// consensus_flag (consensus_helper.py:509-565).
template <typename Get>
__device__ int32_t serial_mode(int32_t beg, int32_t end, const uint4* __restrict__ meta, Get get, bool is_flag) {
    int32_t best_cnt = -1, best_val = 0, nmax = 0;
    for (int32_t j = beg; j < end; ++j) {
        const uint4 mj = meta[j];
        if (!((mj.w >> 23) & 1u)) continue;
        const int32_t v = get(j, mj);
        bool first = true;
        for (int32_t k = beg; k < j && first; ++k) {
            const uint4 mk = meta[k];
            if (((mk.w >> 23) & 1u) && get(k, mk) == v) first = false;
        }
        if (!first) continue;
        int32_t c = 0;
        for (int32_t k = j; k < end; ++k) {
            const uint4 mk = meta[k];
            if (((mk.w >> 23) & 1u) && get(k, mk) == v) ++c;
        }
        if (c > best_cnt) { best_cnt = c; best_val = v; nmax = 1; }
        else if (c == best_cnt) ++nmax;
    }
    if (!is_flag || nmax == 1) return best_val;
    const int32_t pri[4] = {99, 83, 147, 163};
    for (int pi = 0; pi < 4; ++pi) {
        int32_t c = 0;
        for (int32_t k = beg; k < end; ++k) {
            const uint4 mk = meta[k];
            if (((mk.w >> 23) & 1u) && get(k, mk) == pri[pi]) ++c;
        }
        if (c == best_cnt) return pri[pi];
    }
    return best_val;
}

// The same mode in one pass over the members (4 loads in flight) with the distinct values kept in
// first-seen order in registers: false when the family holds more than MODE_K distinct values (the
// caller then takes serial_mode).  Ties: the first-seen maximum, for flags the priority above.
constexpr int MODE_K = 4;
template <typename Get>
__device__ bool table_mode(int32_t cnt, const uint4* __restrict__ fm, Get get, bool is_flag, int32_t& out) {
    int32_t val[MODE_K], num[MODE_K];
    int nv = 0;
#pragma unroll
    for (int i = 0; i < MODE_K; ++i) { val[i] = 0; num[i] = 0; }
    for (int32_t k0 = 0; k0 < cnt; k0 += 4) {
        uint4 mm[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) mm[u] = k0 + u < cnt ? fm[k0 + u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!((mm[u].w >> 23) & 1u)) continue;
            const int32_t v = get(mm[u]);
            bool hit = false;
#pragma unroll
            for (int i = 0; i < MODE_K; ++i)
                if (i < nv && val[i] == v) { ++num[i]; hit = true; }
            if (hit) continue;
            if (nv == MODE_K) return false;
#pragma unroll
            for (int i = 0; i < MODE_K; ++i)
                if (i == nv) { val[i] = v; num[i] = 1; }
            ++nv;
        }
    }
    int32_t best_cnt = -1, best_val = 0, nmax = 0;
#pragma unroll
    for (int i = 0; i < MODE_K; ++i) {
        if (i >= nv) continue;
        if (num[i] > best_cnt) { best_cnt = num[i]; best_val = val[i]; nmax = 1; }
        else if (num[i] == best_cnt) ++nmax;
    }
    out = best_val;
    if (!is_flag || nmax == 1) return true;
    const int32_t pri[4] = {99, 83, 147, 163};
    for (int pi = 0; pi < 4; ++pi) {
        int32_t c = 0;
#pragma unroll
        for (int i = 0; i < MODE_K; ++i)
            if (i < nv && val[i] == pri[pi]) c = num[i];
        if (c == best_cnt) { out = pri[pi]; return true; }
    }
    return true;
}

struct SwarWord {
    uint32_t pc, ca, cc, cg, orb, ql;
};

// bytes with bit 7 set -> 0xff, others 0
__device__ __forceinline__ uint32_t ff_of_80(uint32_t m80) { return (m80 - (m80 >> 7)) | m80; }

__device__ __forceinline__ uint32_t min60_bytes(uint32_t q) {
    const uint32_t hi = ff_of_80((((q | 0x80808080u) - 0x3d3d3d3du) | q) & 0x80808080u);   // q > 60
    return (hi & 0x3c3c3c3cu) | (~hi & q);
}

__device__ __forceinline__ void swar_member(SwarWord& s, uint32_t w, uint32_t q) {
    // q >= 30 per byte: (q | 0x80) - 30 keeps bit 7 iff q >= 30 for q < 128; OR-ing q back keeps
    // q >= 128 passing.  No byte borrows: every byte of (q | 0x80) is >= 0x80.
    const uint32_t p80 = (((q | 0x80808080u) - 0x1e1e1e1eu) | q) & 0x80808080u;
    const uint32_t p1 = p80 >> 7;
    const uint32_t pff = (p80 - p1) | p80;
    s.pc += p1;
    s.ql = (q & pff) | (s.ql & ~pff);
    const uint32_t wp = w & pff;
    s.orb |= wp;
    s.ca += wp & 0x01010101u;
    s.cc += wp & 0x02020202u;
    s.cg += wp & 0x04040404u;
}

// Vote planner, one thread per emitted family (SSCS_maker.py:312-339 order): assigns the vote slot,
// checks every member once (short read, missing qualities, missing cigar, bases outside ACGTN)
// and resolves the create_aligned_segment fields (consensus_helper.py:509-619): member 0's value
// unless the family disagrees, then the exact mode.  Families the SWAR vote cannot take (more than
// VOTE_BIGN members, or all with all_slow) go to the split vote through a device-counted list;
// that kernel reports their errors and fields itself.  vote_order[] = {first member, members incl.
// dropped (0: handed over), consensus length L, vote slot}, ordered by member count per block.
__global__ __launch_bounds__(256) void k_vote_plan(
    int64_t n, const uint8_t* __restrict__ needv, const uint32_t* __restrict__ vx, const int32_t* __restrict__ emit_fam,
    const int2* __restrict__ emit_span, const uint4* __restrict__ mem_meta,
    const int32_t* __restrict__ mem_rec, DevTable T, int32_t* __restrict__ vote_fam, int4* __restrict__ vote_order,
    int32_t* __restrict__ emit_vslot, int32_t* __restrict__ out_meta, uint32_t* __restrict__ slow_n,
    int32_t* __restrict__ slow_list, uint32_t* __restrict__ n_items, int all_slow, uint32_t* __restrict__ err) {
    __shared__ uint32_t s_bin[64], s_cur[64];
    __shared__ int64_t s_vb;
    const int tid = threadIdx.x;
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + tid;
    int4 rec = make_int4(0, 0, 0, -1);
    int key = -1;                                            // bin of this thread's vote slot, -1: none
    uint32_t eb = 0;
    if (o < n) {
        if (!needv[o]) {
            emit_vslot[o] = -1;
        } else {
            const int32_t f = emit_fam[o];
            const int32_t v = (int32_t)vx[o];
            vote_fam[v] = f;
            emit_vslot[o] = v;
            const int2 sp = emit_span[o];
            const int32_t beg = sp.x, cnt = sp.y;
            const uint4* fm = mem_meta + beg;
            const uint4 m0 = fm[0];
            const uint32_t ql0 = m0.z >> 16;
            const int32_t L = ql0 == 0xffffu ? -1 : (int32_t)ql0;   // infer_query_length of member 0 (Q5)
            uint32_t d = 0;
            const bool slow = cnt > VOTE_BIGN || all_slow;
            // the split vote checks its families' members itself: no walk over them here
            for (int32_t k0 = 0; !slow && k0 < cnt; k0 += 4) {
                uint4 mm[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) mm[u] = k0 + u < cnt ? fm[k0 + u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint4 m = mm[u];
                    if (!((m.w >> 23) & 1u)) continue;       // dropped ("line read twice") or past the end
                    const uint32_t ls = m.z & 0xffffu;
                    if (L < 0) eb |= EB_NO_CIGAR;
                    else if ((int32_t)ls < L) eb |= EB_SHORT;
                    if (((m.w >> 20) & CC_RF_QUAL_MISSING) && L > 0) eb |= EB_NO_QUAL;
                    if (((m.w >> 12) & 0xffu) != ((m0.w >> 12) & 0xffu)) d |= 1u;
                    if (m.y != m0.y) d |= 2u;
                    if ((m.w & 0xfffu) != (m0.w & 0xfffu)) d |= 4u;
                    const uint32_t rg7 = (m.w >> 24) & 0x7fu;
                    const bool badrg = ((m.w >> 20) & CC_RF_RG_UNSUPPORTED) != 0;
                    if (rg7 != ((m0.w >> 24) & 0x7fu)) d |= 8u;
                    if (rg7 == 0x7eu) d |= 64u;
                    if (rg7 == 0x7fu && !badrg) d |= 16u;
                    if (badrg) d |= 32u;
                }
            }
            key = 0;
            rec = make_int4(beg, 0, 0, v);
            if (slow) {
                slow_list[atomicAdd(slow_n, 1u)] = v;
                if (cnt > BIG_CH) atomicAdd(n_items, (uint32_t)((cnt + BIG_CH - 1) / BIG_CH));
                eb = 0;                                      // the exact kernel reports this family
            } else {
                int32_t mapq = (int32_t)((m0.w >> 12) & 0xffu), tlen = (int32_t)m0.y, flag = (int32_t)(m0.w & 0xfffu);
                const auto g_mapq = [](const uint4& m) { return (int32_t)((m.w >> 12) & 0xffu); };
                const auto g_tlen = [](const uint4& m) { return (int32_t)m.y; };
                const auto g_flag = [](const uint4& m) { return (int32_t)(m.w & 0xfffu); };
                if ((d & 1u) && !table_mode(cnt, fm, g_mapq, false, mapq))
                    mapq = serial_mode(0, cnt, fm, [&](int32_t, const uint4& m) { return g_mapq(m); }, false);
                if ((d & 2u) && !table_mode(cnt, fm, g_tlen, false, tlen))
                    tlen = serial_mode(0, cnt, fm, [&](int32_t, const uint4& m) { return g_tlen(m); }, false);
                if ((d & 4u) && !table_mode(cnt, fm, g_flag, true, flag))
                    flag = serial_mode(0, cnt, fm, [&](int32_t, const uint4& m) { return g_flag(m); }, true);
                // RG: any member without RG makes get_tag raise -> no RG (consensus_helper.py:614-617)
                int32_t rg = -1;
                if (!(d & 16u)) {
                    if (d & 32u) eb |= EB_RG;
                    else if (!(d & (8u | 64u))) rg = (int32_t)((m0.w >> 24) & 0x7fu);
                    else rg = serial_mode(0, cnt, fm, [&](int32_t j, const uint4& m) {
                        const uint32_t r7 = (m.w >> 24) & 0x7fu;
                        return r7 == 0x7eu ? T.rg[mem_rec[beg + j]] : (int32_t)r7; }, false);
                }
                const int32_t Lp = L < 0 ? 0 : L;
                out_meta[5 * v + 0] = Lp;
                out_meta[5 * v + 1] = mapq;
                out_meta[5 * v + 2] = tlen;
                out_meta[5 * v + 3] = flag;
                out_meta[5 * v + 4] = rg;
                rec = make_int4(beg, cnt, Lp, v);
                key = cnt;
            }
        }
    }
    if (eb) atomicOr(err, eb);
    // The block's vote slots are one contiguous range (vx is an exclusive scan); lay its families out
    // in member-count order there (counting sort in LDS), so each wave of the vote gets families of
    // about the same size and its member loop runs about as long for every lane.
    if (tid < 64) s_bin[tid] = 0u;
    if (tid == 0) s_vb = (int64_t)blockIdx.x * blockDim.x < n ? (int64_t)vx[(int64_t)blockIdx.x * blockDim.x] : 0;
    __syncthreads();
    if (key >= 0) atomicAdd(&s_bin[key], 1u);
    __syncthreads();
    if (tid < 64) {
        const uint32_t c = s_bin[tid];
        uint32_t x = c;
#pragma unroll
        for (int d2 = 1; d2 < 64; d2 <<= 1) {
            const uint32_t y = __shfl_up(x, d2, 64);
            if (tid >= d2) x += y;
        }
        s_cur[tid] = x - c;
    }
    __syncthreads();
    if (key >= 0) vote_order[s_vb + atomicAdd(&s_cur[key], 1u)] = rec;
}

// count[best] == 1 < pass: the quality of the one passing (q >= 30) member whose base at
// position i is `code`, capped at 60 (SSCS_maker.py:134-144).  Rare; kept out of line.
__device__ __noinline__ uint32_t lone_quality(const uint4* __restrict__ fm, int32_t cnt, int32_t i, uint32_t code,
                                              const uint8_t* __restrict__ payload) {
    uint32_t qs = 0;
    for (int32_t k = 0; k < cnt; ++k) {
        const uint4 mk = fm[k];
        const uint32_t lsk = mk.z & 0xffffu;
        if (!((mk.w >> 23) & 1u) || i >= (int32_t)lsk) continue;
        const uint64_t qok = (uint64_t)mk.x << 4;
        const uint32_t qq = payload[qok + i];
        const uint32_t by = payload[qok + ((lsk + 15u) & ~15u) + (i >> 1)];
        const uint32_t b = (i & 1) ? (by & 15u) : (by >> 4);
        if (qq >= 30u && b == code) qs += qq;
    }
    return qs > 60u ? 60u : qs;
}

// a member with q >= 30 and an N at position i (orb 15 there: a passing N, or A, C, G and T all
// passing).  Rare; kept out of line.
__device__ __noinline__ bool passing_n(const uint4* __restrict__ fm, int32_t cnt, int32_t i,
                                       const uint8_t* __restrict__ payload) {
    for (int32_t k = 0; k < cnt; ++k) {
        const uint4 mk = fm[k];
        const uint32_t lsk = mk.z & 0xffffu;
        if (!((mk.w >> 23) & 1u) || i >= (int32_t)lsk) continue;
        const uint64_t qok = (uint64_t)mk.x << 4;
        const uint32_t by = payload[qok + ((lsk + 15u) & ~15u) + (i >> 1)];
        const uint32_t b = (i & 1) ? (by & 15u) : (by >> 4);
        if (payload[qok + i] >= 30u && b == 15u) return true;
    }
    return false;
}

// The vote proper: lane = (family, 16-position chunk), fpw families per wave in vote-slot order.
// Per member one 16-B quality load and one 8-B nibble load; everything else (fields, checks) was
// settled by k_vote_plan, so the loop is loads + byte-sliced counting only.
__global__ __launch_bounds__(256, CC_SV_WAVES) void k_sscs_vote_swar(
    int64_t nv, int32_t fpw, int32_t chunks, const int4* __restrict__ vote_order, const uint4* __restrict__ mem_meta,
    DevTable T, const int32_t* __restrict__ thr, int32_t uni_ok, int32_t qstride, uint8_t* __restrict__ out_seq,
    uint8_t* __restrict__ out_qual, uint32_t* __restrict__ err) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int g = lane / chunks, c = lane - g * chunks;
    const int64_t t = wave * fpw + g;
    int32_t beg = 0, cnt = 0, L = 0;
    int64_t v = 0;
    if (g < fpw && t < nv) {
        const int4 vi = vote_order[t];                  // {first member, members, L, vote slot}
        beg = vi.x; cnt = vi.y; L = vi.z; v = vi.w;
    }
    const int32_t i0 = SV_POS * c;
    uint32_t eb = 0;
    // every lane of a family runs the member loop (its record loads feed the family's shuffles);
    // lanes past the consensus length load nothing and write nothing
    const bool act = i0 < L;
    if (cnt > 0) {
        uint32_t lm[4];
        {
            uint32_t lp[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int32_t rem = L - i0 - 4 * k;
                lp[k] = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : ((1u << (8 * rem)) - 1u));
            }
            lm[0] = __builtin_amdgcn_perm(lp[1], lp[0], 0x06040200u);
            lm[1] = __builtin_amdgcn_perm(lp[1], lp[0], 0x07050301u);
            lm[2] = __builtin_amdgcn_perm(lp[3], lp[2], 0x06040200u);
            lm[3] = __builtin_amdgcn_perm(lp[3], lp[2], 0x07050301u);
        }
        SwarWord s[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) s[k] = SwarWord{};
        const uint4* fm = mem_meta + beg;
        // the nibbles of this lane's positions below L: a base outside A,C,G,T,N there (any member,
        // any quality) is the reference's ValueError (SSCS_maker.py:122,127)
        const int nbl = L - i0 < 16 ? (L - i0 > 0 ? L - i0 : 0) : 16;
        const uint32_t irx = nib_mask(nbl, 0), iry = nib_mask(nbl, 1);
        uint32_t irr = 0;
        // Loads are unconditional (no branches per member): a member past the family, a dropped
        // one or one shorter than this chunk is read at a clamped, valid address and its qualities
        // masked to 0, and a quality of 0 contributes nothing to any counter.
        // The family's member records are fetched chunks at a time, one per lane of the family, and
        // broadcast with lane shuffles: the payload loads of a batch then depend on one record load
        // instead of each member's own (the families of a wave have their lanes side by side).
        const int gl = g * chunks;
        for (int32_t k0 = 0; k0 < cnt; k0 += chunks) {
            const uint4 mine = (k0 + c < cnt) ? fm[k0 + c] : make_uint4(0u, 0u, 0u, 0u);
            const int kn = cnt - k0 < chunks ? cnt - k0 : chunks;
            for (int u0 = 0; u0 < kn; u0 += SV_U) {
                uint4 qv[SV_U];
                uint2 sv[SV_U];
                uint32_t vm[SV_U];
#pragma unroll
                for (int u = 0; u < SV_U; ++u) {
                    const int src = gl + (u0 + u < kn ? u0 + u : kn - 1);
                    const uint32_t mx = (uint32_t)__shfl((int)mine.x, src);
                    const uint32_t mz = (uint32_t)__shfl((int)mine.z, src);
                    const uint32_t mw = (uint32_t)__shfl((int)mine.w, src);
                    const uint32_t ls = mz & 0xffffu;
                    const bool ok = act & (u0 + u < kn) & (((mw >> 23) & 1u) != 0u) & (i0 < (int32_t)ls);
                    vm[u] = ok ? 0xffffffffu : 0u;
                    const uint32_t off = ok ? (uint32_t)i0 : 0u;
                    const uint8_t* base = T.payload + CC_IDX((uint64_t)mx << 4, T.pay_bytes + 1, DS_PAYLOAD);
                    qv[u] = *reinterpret_cast<const uint4*>(base + off);
                    sv[u] = *reinterpret_cast<const uint2*>(base + ((ls + 15u) & ~15u) + (off >> 1));
                }
#pragma unroll
                for (int u = 0; u < SV_U; ++u) {
                    const uint4 q = qv[u];
                    const uint2 sq = sv[u];
                    const uint32_t v = vm[u];
                    irr |= nib_irregular(sq.x, irx & v) | nib_irregular(sq.y, iry & v);
                    swar_member(s[0], (sq.x >> 4) & 0x0f0f0f0fu, __builtin_amdgcn_perm(q.y, q.x, 0x06040200u) & lm[0] & v);
                    swar_member(s[1], sq.x & 0x0f0f0f0fu, __builtin_amdgcn_perm(q.y, q.x, 0x07050301u) & lm[1] & v);
                    swar_member(s[2], (sq.y >> 4) & 0x0f0f0f0fu, __builtin_amdgcn_perm(q.w, q.z, 0x06040200u) & lm[2] & v);
                    swar_member(s[3], sq.y & 0x0f0f0f0fu, __builtin_amdgcn_perm(q.w, q.z, 0x07050301u) & lm[3] & v);
                }
            }
        }
        if (irr) eb |= EB_BAD_BASE;
        uint32_t code[4], qo[4], multi = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const SwarWord& x = s[w];
            // unanimous form: count[best] = pc = pass, so the cutoff holds iff 1.0 >= cutoff
            const uint32_t z80 = ~((x.pc | 0x80808080u) - 0x01010101u) & 0x80808080u;   // pc == 0
            const uint32_t z15 = (z80 >> 3) - (z80 >> 7);
            code[w] = uni_ok ? (x.orb | z15) : 0x0f0f0f0fu;
            const uint32_t g2 = ff_of_80(((x.pc | 0x80808080u) - 0x02020202u) & 0x80808080u);   // pc >= 2
            qo[w] = (g2 & 0x3c3c3c3cu) | (~g2 & min60_bytes(x.ql));
            // positions whose passing members disagree (or a passing N): bit 4w + j
            const uint32_t mu = x.orb & ((x.orb | 0x80808080u) - 0x01010101u) & lm[w];
            const uint32_t mb = ((mu | (mu >> 1) | (mu >> 2) | (mu >> 3)) & 0x01010101u) * 0x01020408u;
            multi |= (mb >> 24) << (4 * w);
        }
#pragma unroll 1
        while (multi) {
            // per position: first maximum of A,C,G,T; the exact cutoff through thr[]
            const int bit = __ffs(multi) - 1;
            multi &= multi - 1u;
            const int w = bit >> 2, j = bit & 3;
            const uint32_t sh = 8u * j;
            // field selects by value: an indexed s[w] would put the accumulators in scratch
#define SV_SEL4(f) (w == 0 ? s[0].f : w == 1 ? s[1].f : w == 2 ? s[2].f : s[3].f)
            const uint32_t xca = SV_SEL4(ca), xcc = SV_SEL4(cc), xcg = SV_SEL4(cg), xpc = SV_SEL4(pc), xql = SV_SEL4(ql),
                           xorb = SV_SEL4(orb);
#undef SV_SEL4
            const int32_t a = (int32_t)((xca >> sh) & 0xffu);
            const int32_t cC = (int32_t)(((xcc >> sh) & 0xffu) >> 1);
            const int32_t gG = (int32_t)(((xcg >> sh) & 0xffu) >> 2);
            const int32_t pass = (int32_t)((xpc >> sh) & 0xffu);   // len(readList) - phred_fail
            const int32_t tT = pass - a - cC - gG;   // garbage only beside a passing N (error)
            const int32_t pos = i0 + 8 * (w >> 1) + 2 * j + (w & 1);
            if (((xorb >> sh) & 0xffu) == 15u && passing_n(fm, cnt, pos, T.payload)) eb |= EB_N_HIGHQ;
            int32_t best = a, mbase = 0;
            if (cC > best) { best = cC; mbase = 1; }
            if (gG > best) { best = gG; mbase = 2; }
            if (tT > best) { best = tT; mbase = 3; }
            const uint32_t cj = (pass > 0 && best >= thr[pass]) ? (1u << mbase) : 15u;
            uint32_t qj;
            if (best >= 2) qj = 60u;
            else if (best <= 0) qj = 0u;
            else if (pass == 1) { const uint32_t qq = (xql >> sh) & 0xffu; qj = qq > 60u ? 60u : qq; }
            else qj = lone_quality(fm, cnt, pos, 1u << mbase, T.payload);
            const uint32_t keep = ~(0xffu << sh);
            if (w == 0) { code[0] = (code[0] & keep) | (cj << sh); qo[0] = (qo[0] & keep) | (qj << sh); }
            else if (w == 1) { code[1] = (code[1] & keep) | (cj << sh); qo[1] = (qo[1] & keep) | (qj << sh); }
            else if (w == 2) { code[2] = (code[2] & keep) | (cj << sh); qo[2] = (qo[2] & keep) | (qj << sh); }
            else { code[3] = (code[3] & keep) | (cj << sh); qo[3] = (qo[3] & keep) | (qj << sh); }
        }
        // back to position order: bytes (E0, O0, E1, O1) and (E2, O2, E3, O3); positions >= L zero
        if (act) {
        uint4 qout;
        qout.x = __builtin_amdgcn_perm(qo[1] & lm[1], qo[0] & lm[0], 0x05010400u);
        qout.y = __builtin_amdgcn_perm(qo[1] & lm[1], qo[0] & lm[0], 0x07030602u);
        qout.z = __builtin_amdgcn_perm(qo[3] & lm[3], qo[2] & lm[2], 0x05010400u);
        qout.w = __builtin_amdgcn_perm(qo[3] & lm[3], qo[2] & lm[2], 0x07030602u);
        *reinterpret_cast<uint4*>(out_qual + v * (int64_t)qstride + i0) = qout;
        *reinterpret_cast<uint2*>(out_seq + v * (int64_t)(qstride >> 1) + (i0 >> 1)) =
            make_uint2(((code[0] & lm[0]) << 4) | (code[1] & lm[1]), ((code[2] & lm[2]) << 4) | (code[3] & lm[3]));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) eb |= __shfl_xor(eb, o);
    if (lane == 0 && eb) atomicOr(err, eb);
}

// The items of the large families (k_big_items): exactly k_sscs_vote_swar's member loop over one
// chunk of at most BIG_CH members, lane = 16 positions (every chunks-th 16 when reads are longer
// than 64 lanes), fpw items per wave; the byte counters go out as four planes in position order.
// Bases outside A,C,G,T,N and a passing N are detected here, per chunk.
__global__ __launch_bounds__(256) void k_big_swar(const uint32_t* __restrict__ d_items, int64_t cap, int32_t fpw,
                                                  int32_t chunks, const int4* __restrict__ items,
                                                  const uint4* __restrict__ mem_meta, DevTable T, int32_t lp,
                                                  uint8_t* __restrict__ partial, uint32_t* __restrict__ err) {
    // the wave's items' member records staged in LDS first (reads of up to BIG_STAGE items per wave,
    // 150-bp reads and longer): the member loop then waits on LDS, not on a global load, before each
    // member's payload loads
    __shared__ uint4 s_meta[4][BIG_STAGE][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const int g = lane / chunks, c = lane - g * chunks;
    const int64_t t = wave * fpw + g;
    const int64_t ni = min((int64_t)*d_items, cap);
    int32_t cnt = 0, L = 0;
    const uint4* fm = mem_meta;
    uint8_t* out = partial;
    if (g < fpw && t < ni) {
        const int4 it = items[t];                  // {vote slot, family's first member, chunk start, chunk size}
        L = big_len(mem_meta[it.y], T.max_len);
        fm = mem_meta + it.z;
        cnt = it.w;
        out = partial + t * (int64_t)BIG_PL * lp;
    }
    if (fpw <= BIG_STAGE) {   // (uniform: a kernel argument)
#pragma unroll 1
        for (int j = 0; j < fpw; ++j) {
            const int64_t tj = wave * fpw + j;
            uint4 mv = make_uint4(0u, 0u, 0u, 0u);
            if (tj < ni) {
                const int4 itj = items[tj];
                if (lane < itj.w) mv = mem_meta[itj.z + lane];
            }
            s_meta[wv][j][lane] = mv;
        }
        __syncthreads();
    }
    const bool staged = fpw <= BIG_STAGE;
    const uint4* sm = &s_meta[wv][g < BIG_STAGE ? g : 0][0];
    uint32_t eb = 0;
    for (int32_t i0 = SV_POS * c; cnt > 0 && i0 < L; i0 += SV_POS * chunks) {
        uint32_t lm[4];
        {
            uint32_t lp4[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int32_t rem = L - i0 - 4 * k;
                lp4[k] = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : ((1u << (8 * rem)) - 1u));
            }
            lm[0] = __builtin_amdgcn_perm(lp4[1], lp4[0], 0x06040200u);
            lm[1] = __builtin_amdgcn_perm(lp4[1], lp4[0], 0x07050301u);
            lm[2] = __builtin_amdgcn_perm(lp4[3], lp4[2], 0x06040200u);
            lm[3] = __builtin_amdgcn_perm(lp4[3], lp4[2], 0x07050301u);
        }
        SwarWord s[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) s[k] = SwarWord{0u, 0u, 0u, 0u, 0u, 0u};
        const int nbl = L - i0 < 16 ? (L - i0 > 0 ? L - i0 : 0) : 16;
        const uint32_t irx = nib_mask(nbl, 0), iry = nib_mask(nbl, 1);
        uint32_t irr = 0;
        for (int32_t k0 = 0; k0 < cnt; k0 += BIG_U) {
            uint4 qv[BIG_U];
            uint2 sv[BIG_U];
            uint32_t vm[BIG_U];
#pragma unroll
            for (int u = 0; u < BIG_U; ++u) {
                const int32_t k = k0 + u < cnt ? k0 + u : cnt - 1;
                const uint4 m = staged ? sm[k] : fm[k];
                const uint32_t ls = m.z & 0xffffu;
                const bool ok = (k0 + u < cnt) & (((m.w >> 23) & 1u) != 0u) & (i0 < (int32_t)ls);
                vm[u] = ok ? 0xffffffffu : 0u;
                const uint32_t off = ok ? (uint32_t)i0 : 0u;
                const uint8_t* base = T.payload + ((uint64_t)m.x << 4);
                qv[u] = *reinterpret_cast<const uint4*>(base + off);
                sv[u] = *reinterpret_cast<const uint2*>(base + ((ls + 15u) & ~15u) + (off >> 1));
            }
#pragma unroll
            for (int u = 0; u < BIG_U; ++u) {
                const uint4 q = qv[u];
                const uint2 sq = sv[u];
                const uint32_t v = vm[u];
                irr |= nib_irregular(sq.x, irx & v) | nib_irregular(sq.y, iry & v);
                swar_member(s[0], (sq.x >> 4) & 0x0f0f0f0fu, __builtin_amdgcn_perm(q.y, q.x, 0x06040200u) & lm[0] & v);
                swar_member(s[1], sq.x & 0x0f0f0f0fu, __builtin_amdgcn_perm(q.y, q.x, 0x07050301u) & lm[1] & v);
                swar_member(s[2], (sq.y >> 4) & 0x0f0f0f0fu, __builtin_amdgcn_perm(q.w, q.z, 0x06040200u) & lm[2] & v);
                swar_member(s[3], sq.y & 0x0f0f0f0fu, __builtin_amdgcn_perm(q.w, q.z, 0x07050301u) & lm[3] & v);
            }
        }
        if (irr) eb |= EB_BAD_BASE;
        // a passing N (orb 15 at a position): the reference's IndexError (SSCS_maker.py:129)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t x = (s[w].orb & lm[w]) ^ 0x0f0f0f0fu;                          // bytes <= 15
            uint32_t hit = ~((x | 0x80808080u) - 0x01010101u) & 0x80808080u;              // orb byte == 15
            while (hit) {
                const int j = (__ffs(hit) - 1) >> 3;
                hit &= hit - 1u;
                const int32_t pos = i0 + 8 * (w >> 1) + 2 * j + (w & 1);
                if (passing_n(fm, cnt, pos, T.payload)) eb |= EB_N_HIGHQ;
            }
        }
        // the four counter planes back in position order (bytes past L are zero through lm)
#define BIG_PLANE(P, FIELD)                                                                                     \
        {                                                                                                       \
            const uint32_t e0 = s[0].FIELD & lm[0], o0 = s[1].FIELD & lm[1];                                    \
            const uint32_t e1 = s[2].FIELD & lm[2], o1 = s[3].FIELD & lm[3];                                    \
            *reinterpret_cast<uint4*>(out + (P) * lp + i0) =                                                    \
                make_uint4(__builtin_amdgcn_perm(o0, e0, 0x05010400u), __builtin_amdgcn_perm(o0, e0, 0x07030602u), \
                           __builtin_amdgcn_perm(o1, e1, 0x05010400u), __builtin_amdgcn_perm(o1, e1, 0x07030602u)); \
        }
        BIG_PLANE(0, pc)
        BIG_PLANE(1, ca)
        BIG_PLANE(2, cc)
        BIG_PLANE(3, cg)
#undef BIG_PLANE
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) eb |= __shfl_xor(eb, o);
    if (lane == 0 && eb) atomicOr(err, eb);
}

__global__ __launch_bounds__(64) void k_big_final(const uint32_t* __restrict__ d_nbig, const int32_t* __restrict__ slow_list,
                                                  const int32_t* __restrict__ big_item, int64_t cap,
                                                  const int32_t* __restrict__ vote_fam,
                                                  const int32_t* __restrict__ fam_beg, const int32_t* __restrict__ fam_end,
                                                  const int32_t* __restrict__ fam_n, const int32_t* __restrict__ mem_rec,
                                                  const uint32_t* __restrict__ mem_valid,
                                                  const uint4* __restrict__ mem_meta, DevTable T, double cutoff,
                                                  int32_t lp, const uint8_t* __restrict__ partial, int32_t qstride,
                                                  uint8_t* __restrict__ out_seq, uint8_t* __restrict__ out_qual,
                                                  int32_t* __restrict__ out_meta, uint32_t* __restrict__ err) {
    __shared__ int32_t s_key[MODE_SLOTS];
    __shared__ uint32_t s_cnt[MODE_SLOTS], s_first[MODE_SLOTS];
    const int lane = threadIdx.x;
    const int64_t nb = (int64_t)*d_nbig;
    for (int64_t k = blockIdx.x; k < nb; k += gridDim.x) {
        const int64_t w = slow_list[k];
        const int32_t item0 = big_item[k];          // first work item (families of one chunk: none)
        const int32_t f = vote_fam[w];
        const int32_t beg = fam_beg[f], end = fam_end[f];
        const int32_t n = fam_n[f];
        const int32_t nch = item0 < 0 ? 1 : (end - beg + BIG_CH - 1) / BIG_CH;
        const uint4 m0 = mem_meta[beg];
        const uint32_t ql0 = m0.z >> 16;
        int32_t L = (int32_t)ql0;
        uint32_t eb = 0;
        if (ql0 == 0xffffu) { eb |= EB_NO_CIGAR; L = 0; }
        if (L > T.max_len) { eb |= EB_SHORT; L = 0; }
        // members: checks and "does every one carry member 0's value" per mode field
        bool d_mapq = false, d_tlen = false, d_flag = false, d_rg = false, rg_missing = false, rg_bad = false;
        // (8 member records in flight per lane: a family of thousands is 8x fewer load round trips)
        constexpr int BM = 8;
        for (int32_t jb = beg; jb < end; jb += 64 * BM) {
            uint4 mm[BM];
#pragma unroll
            for (int u = 0; u < BM; ++u) {
                const int32_t j = jb + 64 * u + lane;
                mm[u] = j < end ? mem_meta[j] : make_uint4(0u, 0u, 0u, 0u);   // w bit 23 clear: skipped
            }
#pragma unroll
            for (int u = 0; u < BM; ++u) {
            const uint4 m = mm[u];
            if (!((m.w >> 23) & 1u)) continue;
            const uint32_t ls = m.z & 0xffffu;
            if ((int32_t)ls < L) eb |= EB_SHORT;
            if (((m.w >> 20) & CC_RF_QUAL_MISSING) && L > 0) eb |= EB_NO_QUAL;
            d_mapq |= ((m.w >> 12) & 0xffu) != ((m0.w >> 12) & 0xffu);
            d_tlen |= m.y != m0.y;
            d_flag |= (m.w & 0xfffu) != (m0.w & 0xfffu);
            const uint32_t rg7 = (m.w >> 24) & 0x7fu;
            const bool badrg = ((m.w >> 20) & CC_RF_RG_UNSUPPORTED) != 0;
            rg_bad |= badrg;
            rg_missing |= (rg7 == 0x7fu) && !badrg;
            d_rg |= (rg7 != ((m0.w >> 24) & 0x7fu)) || rg7 == 0x7eu;
            }
        }
        // the consensus: a family of one chunk (reads longer than the SWAR lanes) counted here, more
        // summed from k_big_swar's planes
        if (nch > 1 && (int64_t)item0 + nch > cap) L = 0;   // over the planned items: the pass re-runs
        uint8_t* oq = out_qual + w * (int64_t)qstride;
        uint8_t* os = out_seq + w * (int64_t)(qstride >> 1);
        for (int32_t c0 = 0; c0 < L; c0 += 256) {
            const int32_t i0 = c0 + 4 * lane;
            uint32_t cnt[4][4], qs[4][4], fail[4];
            if (nch == 1) {
                big_count(beg, end, L, i0, lane, mem_meta, T, cnt, qs, fail, eb);
            } else {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    fail[t] = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) { cnt[t][b] = 0; qs[t][b] = 0; }
                }
                // (unrolled: the planes of several items in flight per lane)
#pragma unroll 8
                for (int32_t c = 0; c < nch && i0 < L; ++c) {
                    const uint8_t* pp = partial + (int64_t)(item0 + c) * BIG_PL * lp + i0;
                    const uint32_t pc = *reinterpret_cast<const uint32_t*>(pp);
                    const uint32_t ca = *reinterpret_cast<const uint32_t*>(pp + lp);
                    const uint32_t cc = *reinterpret_cast<const uint32_t*>(pp + 2 * lp);
                    const uint32_t cg = *reinterpret_cast<const uint32_t*>(pp + 3 * lp);
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const uint32_t p1 = (pc >> (8 * t)) & 0xffu, a1 = (ca >> (8 * t)) & 0xffu;
                        const uint32_t c1 = ((cc >> (8 * t)) & 0xffu) >> 1, g1 = ((cg >> (8 * t)) & 0xffu) >> 2;
                        cnt[t][0] += a1; cnt[t][1] += c1; cnt[t][2] += g1; cnt[t][3] += p1 - a1 - c1 - g1;
                        fail[t] += p1;   // here: the passing count (pass below)
                    }
                }
            }
            if (i0 >= L) continue;
            uint32_t qout = 0, sout = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                uint32_t code = 0, mq = 0;
                if (i0 + t < L) {
                    int m = 0;
                    uint32_t best = cnt[t][0];
#pragma unroll
                    for (int b = 1; b < 4; ++b)
                        if (cnt[t][b] > best) { best = cnt[t][b]; m = b; }
                    int32_t pass;
                    if (nch == 1) {
                        uint32_t qsm = qs[t][0];
#pragma unroll
                        for (int b = 1; b < 4; ++b)
                            if (m == b) qsm = qs[t][b];
                        mq = qsm > 60u ? 60u : qsm;
                        pass = n - (int32_t)fail[t];
                    } else {
                        pass = (int32_t)fail[t];
                        mq = best >= 2u ? 60u : best == 0u ? 0u
                                                           : lone_quality(mem_meta + beg, end - beg, i0 + t, 1u << m, T.payload);
                    }
                    // nuc_count[max]/phred_pass_reads >= cutoff in IEEE double, as Python evaluates it
                    const bool ok = pass != 0 && ((double)best / (double)pass) >= cutoff;
                    code = ok ? (1u << m) : 15u;
                }
                qout |= mq << (8 * t);
                const int sh = (t == 0) ? 4 : (t == 1) ? 0 : (t == 2) ? 12 : 8;   // position i0 -> high nibble
                sout |= code << sh;
            }
            *reinterpret_cast<uint32_t*>(oq + i0) = qout;
            *reinterpret_cast<uint16_t*>(os + (i0 >> 1)) = (uint16_t)sout;
        }
        d_mapq = __any(d_mapq);
        d_tlen = __any(d_tlen);
        d_flag = __any(d_flag);
        d_rg = __any(d_rg);
        rg_missing = __any(rg_missing);
        rg_bad = __any(rg_bad);
        int32_t mapq = (int32_t)((m0.w >> 12) & 0xffu), tlen = (int32_t)m0.y, flag = (int32_t)(m0.w & 0xfffu);
        bool ovf = false;
        if (d_mapq) {
            mapq = lds_mode(lane, beg, end, mem_meta, [&](int32_t j) { return (int32_t)((mem_meta[j].w >> 12) & 0xffu); },
                            false, s_key, s_cnt, s_first, &ovf);
            if (ovf) mapq = wave_mode(lane, beg, end, mem_rec, mem_valid, [&](int32_t r) { return (int32_t)T.mapq[r]; }, false);
        }
        if (d_tlen) {
            tlen = lds_mode(lane, beg, end, mem_meta, [&](int32_t j) { return (int32_t)mem_meta[j].y; }, false, s_key,
                            s_cnt, s_first, &ovf);
            if (ovf) tlen = wave_mode(lane, beg, end, mem_rec, mem_valid, [&](int32_t r) { return T.tlen[r]; }, false);
        }
        if (d_flag) {
            flag = lds_mode(lane, beg, end, mem_meta, [&](int32_t j) { return (int32_t)(mem_meta[j].w & 0xfffu); }, true,
                            s_key, s_cnt, s_first, &ovf);
            if (ovf) flag = wave_mode(lane, beg, end, mem_rec, mem_valid, [&](int32_t r) { return (int32_t)T.flag[r]; }, true);
        }
        // RG: any member without RG makes get_tag raise -> no RG (consensus_helper.py:614-617)
        int32_t rg = -1;
        if (!rg_missing) {
            if (rg_bad) eb |= EB_RG;
            else if (!d_rg) rg = (int32_t)((m0.w >> 24) & 0x7fu);
            else {
                rg = lds_mode(lane, beg, end, mem_meta, [&](int32_t j) { return T.rg[mem_rec[j]]; }, false, s_key, s_cnt,
                              s_first, &ovf);
                if (ovf) rg = wave_mode(lane, beg, end, mem_rec, mem_valid, [&](int32_t r) { return T.rg[r]; }, false);
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) eb |= __shfl_xor(eb, o);
        if (lane == 0) {
            out_meta[5 * w + 0] = L;
            out_meta[5 * w + 1] = mapq;
            out_meta[5 * w + 2] = tlen;
            out_meta[5 * w + 3] = flag;
            out_meta[5 * w + 4] = rg;
            if (eb) atomicOr(err, eb);
        }
    }
}

// ------------------------------------------------------------------ duplex lookups
// Open-addressing table tag-hash -> family (linear probing).  Family hashes are unique after a
// successful read_bam (equal hashes of different tags abort with CC_E_COLLISION), so a probe
// that meets the hash has found the only candidate; the tag itself is still compared.
__global__ __launch_bounds__(256) void k_ht_insert(int64_t F, const uint64_t* __restrict__ fam_hash,
                                                   unsigned long long* __restrict__ ht_key,
                                                   int32_t* __restrict__ ht_val, uint64_t mask) {
    int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    const unsigned long long h = fam_hash[f];
    uint64_t slot = h & mask;
    while (true) {
        const unsigned long long prev = atomicCAS(&ht_key[slot], ~0ULL, h);
        if (prev == ~0ULL) { ht_val[slot] = (int32_t)f; return; }
        slot = (slot + 1) & mask;
    }
}

__device__ __forceinline__ int32_t lookup_ht(const TagKey& key, uint64_t seed, const unsigned long long* __restrict__ ht_key,
                                             const int32_t* __restrict__ ht_val, uint64_t mask,
                                             const TagKey* __restrict__ fam_tag) {
    const unsigned long long h = hash_tag(key, seed);
    uint64_t slot = h & mask;
    while (true) {
        const unsigned long long k = ht_key[slot];
        if (k == ~0ULL) return -1;
        if (k == h) {
            const int32_t f = ht_val[slot];
            if (tag_eq(fam_tag[f], key)) return f;
        }
        slot = (slot + 1) & mask;
    }
}

// duplex_tag (consensus_helper.py:639-683) on the packed key: swap barcode, R1<->R2 (None -> R1)
__device__ __forceinline__ bool duplex_key(const TagKey& t, const int32_t* __restrict__ bc_swap, int nbc, TagKey& u) {
    u = t;
    if (t.bc < 0 || t.bc >= nbc) return false;
    int32_t sb = bc_swap[t.bc];
    if (sb < 0) return false;
    u.bc = sb;
    uint32_t rn = (t.bits >> 1) & 3u;
    uint32_t nrn = (rn == 0u) ? 1u : 0u;
    u.bits = (t.bits & ~6u) | (nrn << 1);
    return true;
}

struct GroupView {  // device pointers of a read_bam group used by the joins
    int64_t F;
    uint64_t seed;
    const unsigned long long* ht_key;
    const int32_t* ht_val;
    uint64_t ht_mask;
    const uint64_t* fam_hash;
    const int32_t* fam_first;
    const int32_t* fam_beg;
    const int32_t* fam_region;
    const int32_t* fam_o;
    const TagKey* fam_tag;   // per family its tag (k_fam_build)
    const int32_t* fam_rec;  // per family its first member's record (with fam_tag)
    const int32_t* mem_rec;
    const int32_t* ent_f;
    int local;   // 1: coordinate-sorted grouping, every position group's families are contiguous
    // family-bucket index over the table's position buckets (local groupings of another table):
    // fbkt[b] = first family whose (tid, pos) lies in bucket b or later
    const int32_t* fbkt;
    const int64_t* tbase;
    const int32_t* geom;   // [0]: bucket width shift
    int32_t ntid;
};

// family f fills the family buckets from the one after family f-1's through its own (f = F: tail);
// a local grouping lists its families in coordinate order, so the buckets are monotone
__global__ __launch_bounds__(256) void k_fam_bucket(int64_t F, const TagKey* __restrict__ fam_tag,
                                                    const int64_t* __restrict__ tbase,
                                                    int32_t ntid, const int32_t* __restrict__ geom,
                                                    int32_t* __restrict__ fbkt) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f > F) return;
    const int32_t bshift = geom[0];
    const int64_t nb = tbase[ntid];
    int64_t b = nb, bp = -1;
    if (f < F) { const TagKey k = fam_tag[f]; b = bucket_of(tbase, ntid, bshift, k.tid, k.pos); }
    if (f > 0) { const TagKey k = fam_tag[f - 1]; bp = bucket_of(tbase, ntid, bshift, k.tid, k.pos); }
    for (int64_t x = bp + 1; x <= b && x <= nb; ++x) fbkt[x] = (int32_t)f;
}

// The family of tag u in another table's local grouping: the families of u's position bucket
__device__ __forceinline__ int32_t lookup_fam_bucket(const TagKey& u, const GroupView& S) {
    const int64_t nb = S.tbase[S.ntid];
    const int64_t b = bucket_of(S.tbase, S.ntid, S.geom[0], u.tid, u.pos);
    const int64_t lo = S.fbkt[b], hi = b < nb ? (int64_t)S.fbkt[b + 1] : S.F;
    for (int64_t h = lo; h < hi; ++h) {
        const TagKey k = S.fam_tag[h];
        if (tag_eq(k, u)) return (int32_t)h;
    }
    return -1;
}

// The family of tag u within f's own position group: a duplex partner keeps tid and pos
// (duplex_tag only swaps the barcode and R1/R2, consensus_helper.py:639-683), so on a coordinate-
// sorted grouping it sits among f's neighbours with the same (tid, pos); otherwise the hash table.
__device__ __forceinline__ int32_t lookup_fam(const TagKey& u, int32_t f, const GroupView& G) {
    if (!G.local) return lookup_ht(u, G.seed, G.ht_key, G.ht_val, G.ht_mask, G.fam_tag);
    for (int64_t h = (int64_t)f + 1; h < G.F; ++h) {
        const TagKey k = G.fam_tag[h];
        if (k.tid != u.tid || k.pos != u.pos) break;
        if (tag_eq(k, u)) return (int32_t)h;
    }
    for (int64_t h = (int64_t)f - 1; h >= 0; --h) {
        const TagKey k = G.fam_tag[h];
        if (k.tid != u.tid || k.pos != u.pos) break;
        if (tag_eq(k, u)) return (int32_t)h;
    }
    return -1;
}

// duplex_tag of family f's tag, and the family holding it (-1: none)
__device__ __forceinline__ int32_t partner_of(int32_t f, const GroupView& G, const int32_t* __restrict__ bc_swap,
                                              int nbc, TagKey& u) {
    const TagKey t = G.fam_tag[f];
    return duplex_key(t, bc_swap, nbc, u) ? lookup_fam(u, f, G) : -1;
}

// Chains of earlier-processed partners are followed this far (a longer chain is reported as
// unsupported rather than guessed; duplex_tag's barcode rotation gives chains of a few steps).
constexpr int DUPLEX_CHAIN = 32;

// DCS_maker.py:245-282 for any duplex_tag, mutual or not.  Tags are processed in csn order q (the
// entry slot; fam_o per family, never for orphan tags).  For tag t with partner u = duplex_tag(t):
//   u not yet in tag_dict (no family, or created in a later region)   -> sscs.singleton (1)
//   u processed before t and made a DCS (u in duplex_dict)            -> skipped (2)
//   u processed before t as an sscs.singleton (read_dict[u] deleted)  -> the reference's KeyError
//   otherwise (u later, an orphan, or skipped itself)                 -> DCS of t with u (0)
// t's decision needs u's only when u was processed earlier, u's needs its partner's under the same
// condition, and so on: the chain's processing orders strictly decrease, so each thread walks its
// own chain and resolves it from the far end.  A mutual pair is a chain of two.
__global__ __launch_bounds__(256) void k_dcs_decide(int64_t Q, GroupView G, const int32_t* __restrict__ bc_swap,
                                                    int nbc, int32_t* __restrict__ dec, int32_t* __restrict__ t_rec,
                                                    int32_t* __restrict__ p_rec, uint8_t* __restrict__ fl_dcs,
                                                    uint32_t* __restrict__ err) {
    int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= Q) return;
    const int32_t f = G.ent_f[q];
    int32_t d = 3, tr = -1, pr = -1;
    if (f >= 0) {
        tr = G.fam_rec[f];
        // the chain of earlier-processed partners: its length n and its first element c0 (the
        // resolution from the far end needs only the length)
        int32_t c0 = -1;
        int n = 0;
        int32_t x = f, ox = (int32_t)q, g = -1;
        bool present = false;
        while (true) {
            TagKey u;
            g = partner_of(x, G, bc_swap, nbc, u);
            present = g >= 0 && G.fam_region[g] <= G.fam_region[x];
            if (!present || G.fam_o[g] >= ox) break;
            if (n == DUPLEX_CHAIN) { atomicOr(err, EB_CHAIN); break; }
            if (n++ == 0) c0 = g;
            x = g;
            ox = G.fam_o[g];
        }
        // the far end: its partner is absent or processed later
        int32_t dx = present ? 0 : 1;
        for (int i = n - 1; i >= 0; --i) {
            // chain element i (processed before the element preceding it) decided dx
            if (dx == 0) dx = 2;
            else if (dx == 1) { atomicOr(err, EB_KEYERROR); dx = 3; }
            else dx = 0;
        }
        d = dx;
        if (d == 0) pr = G.fam_rec[n > 0 ? c0 : g];
    }
    dec[q] = d;
    t_rec[q] = tr;
    p_rec[q] = pr;
    fl_dcs[q] = d == 0 ? 1 : 0;
}

// singleton_correction.py:278-319 for any duplex_tag.  For singleton tag x (processed at order q,
// region r) with partner y = duplex_tag(x):
//   1  the SSCS family y exists in r's chromosome run, read by region r: correction by the SSCS (an
//      SSCS family is only ever looked up by the one tag whose duplex it is, so nothing else
//      deletes it first);
//   2  else the singleton family y exists (created by region r) and was not deleted before x:
//      correction by the singleton; x completes a mutual correction when y is in correction_dict
//      (y took 2 earlier and did not complete one itself), and both leave singleton_dict;
//   3  else uncorrected.
// y was deleted before x iff it was processed earlier and took 1 or 3, or took 2 and completed.
// As for DCS, x depends on y only when y was processed earlier: a chain with decreasing orders.
__global__ __launch_bounds__(256) void k_sc_decide(int64_t Q, GroupView G, GroupView S,
                                                   const int32_t* __restrict__ region_run,
                                                   const int32_t* __restrict__ bc_swap, int nbc,
                                                   int32_t* __restrict__ dec, int32_t* __restrict__ t_rec,
                                                   int32_t* __restrict__ p_rec, uint8_t* __restrict__ fl_corr,
                                                   uint32_t* __restrict__ err) {
    int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= Q) return;
    const int32_t f = G.ent_f[q];
    int32_t d = 3, tr = -1, pr = -1;
    if (f >= 0) {
        tr = G.fam_rec[f];
        int n = 0;   // length of the chain of earlier-processed partners
        int32_t x = f, ox = (int32_t)q;
        int32_t s0 = -1, g0 = -1;     // t's SSCS / singleton partners
        int32_t dx = 3;
        bool comp = false;
        while (true) {
            const int32_t reg = G.fam_region[x];
            TagKey u;
            int32_t s = -1, g = -1;
            if (duplex_key(G.fam_tag[x], bc_swap, nbc, u)) {
                TagKey us = u;
                us.bits = (u.bits & 7u) | ((uint32_t)region_run[reg] << 3);
                s = S.fbkt ? lookup_fam_bucket(us, S)
                           : lookup_ht(us, S.seed, S.ht_key, S.ht_val, S.ht_mask, S.fam_tag);
                if (s >= 0 && S.fam_region[s] > reg) s = -1;      // not read yet
                g = lookup_fam(u, x, G);
                if (g >= 0 && G.fam_region[g] > reg) g = -1;      // not created yet
            }
            if (n == 0) { s0 = s; g0 = g; }
            if (s >= 0) { dx = 1; break; }
            if (g < 0) { dx = 3; break; }
            if (G.fam_o[g] >= ox) { dx = 2; comp = false; break; }   // y later (or an orphan): present
            if (n == DUPLEX_CHAIN) { atomicOr(err, EB_CHAIN); break; }
            ++n;
            x = g;
            ox = G.fam_o[g];
        }
        for (int i = n - 1; i >= 0; --i) {
            // chain element i decided (dx, comp); the element before it has no SSCS partner
            const bool deleted = dx == 1 || dx == 3 || (dx == 2 && comp);
            if (deleted) { dx = 3; comp = false; }
            else { comp = dx == 2 && !comp; dx = 2; }
        }
        d = dx == 1 ? 0 : dx == 2 ? 1 : 2;
        if (d == 0) pr = S.fam_rec[s0];
        else if (d == 1) pr = G.fam_rec[g0];
    }
    dec[q] = d;
    t_rec[q] = tr;
    p_rec[q] = pr;
    fl_corr[q] = (d == 0 || d == 1) ? 1 : 0;
}

// duplex_consensus: DCS (DCS_maker.py:99-123, sc=0) and SC (singleton_correction.py:61-86, sc=1)
// in the byte-sliced form of k_sscs_vote_swar.  One lane owns one 16-position chunk of one output:
// two 16-B quality loads and two 8-B nibble loads, four 32-bit words of four positions each.
// Per position: equal codes (DCS: any code, N == N included; SC: also both q > 29) give that code
// with min(60, q1 + q2) = min(60, min(q1, 60) + min(q2, 60)) (no byte overflow); otherwise 'N' and
// 0.  Length = read1.query_length; modes over [read1, read2] for DCS, over [read1] for SC
// (create_aligned_segment([read], ...), singleton_correction.py:109).

__device__ __forceinline__ void duplex_word(uint32_t wa, uint32_t wb, uint32_t qa, uint32_t qb, int sc,
                                            uint32_t& code, uint32_t& qual) {
    uint32_t ok = ~(((wa ^ wb) | 0x80808080u) - 0x01010101u) & 0x80808080u;          // equal codes
    if (sc) {
        ok &= (((qa | 0x80808080u) - 0x1e1e1e1eu) | qa) & 0x80808080u;               // q1 >= 30
        ok &= (((qb | 0x80808080u) - 0x1e1e1e1eu) | qb) & 0x80808080u;               // q2 >= 30
    }
    const uint32_t ff = ff_of_80(ok);
    code = (wa & ff) | (0x0f0f0f0fu & ~ff);
    qual = min60_bytes(min60_bytes(qa) + min60_bytes(qb)) & ff;                       // sums <= 120
}

__global__ __launch_bounds__(256) void k_duplex_vote_swar(
    int64_t nv, int sc, int32_t fpw, int32_t chunks, const int4* __restrict__ vpair,
    DevTable TA, DevTable TB, int32_t qstride, uint8_t* __restrict__ out_seq, uint8_t* __restrict__ out_qual,
    int32_t* __restrict__ out_meta, uint32_t* __restrict__ err) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int g = lane / chunks, c = lane - g * chunks;
    const int64_t w = wave * fpw + g;
    uint32_t eb = 0;
    if (g < fpw && w < nv) {
        const int4 vp = vpair[w];   // {read1 record, read2 record, decision, entry} (EmitVotePairs)
        const int32_t a = CC_IDX(vp.x, TA.n, DS_VOTE_REC), b = vp.y;
        // SC: a complement found among the singletons (dec 1) lives in the singleton table
        const bool b_in_a = sc && vp.z == 1;
        const DevTable& TBx = b_in_a ? TA : TB;
        const uint8_t* bpay = TBx.payload;
        const uint4 ma = TA.meta[a], mb = TBx.meta[CC_IDX(b, TBx.n, DS_VOTE_REC)];   // pay16, tlen, lseq | qlen << 16, flag | mapq | rflags | rg7
        const int32_t la = (int32_t)(ma.z & 0xffffu), lb = (int32_t)(mb.z & 0xffffu);
        int32_t L = la;                                                      // read1.query_length
        if (lb < L) { eb |= EB_SHORT; L = 0; }
        if (L > 0 && (((ma.w | mb.w) >> 20) & CC_RF_QUAL_MISSING)) eb |= EB_NO_QUAL;
        // reads longer than 64 chunks: each lane takes every chunks-th chunk
        for (int32_t i0 = SV_POS * c; i0 < L; i0 += SV_POS * chunks) {
            const uint64_t qa = (uint64_t)ma.x << 4, qb = (uint64_t)mb.x << 4;
            const uint64_t sa = qa + (uint64_t)((la + 15) & ~15), sb = qb + (uint64_t)((lb + 15) & ~15);
            const uint4 QA = *reinterpret_cast<const uint4*>(TA.payload + qa + i0);
            const uint4 QB = *reinterpret_cast<const uint4*>(bpay + qb + i0);
            const uint2 SA = *reinterpret_cast<const uint2*>(TA.payload + sa + (i0 >> 1));
            const uint2 SB = *reinterpret_cast<const uint2*>(bpay + sb + (i0 >> 1));
            uint32_t lp[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int32_t rem = L - i0 - 4 * k;
                lp[k] = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : ((1u << (8 * rem)) - 1u));
            }
            const uint4 QM = make_uint4(QA.x & lp[0], QA.y & lp[1], QA.z & lp[2], QA.w & lp[3]);
            const uint4 QN = make_uint4(QB.x & lp[0], QB.y & lp[1], QB.z & lp[2], QB.w & lp[3]);
            uint32_t code[4], qo[4];
            duplex_word((SA.x >> 4) & 0x0f0f0f0fu, (SB.x >> 4) & 0x0f0f0f0fu,
                        __builtin_amdgcn_perm(QM.y, QM.x, 0x06040200u), __builtin_amdgcn_perm(QN.y, QN.x, 0x06040200u),
                        sc, code[0], qo[0]);
            duplex_word(SA.x & 0x0f0f0f0fu, SB.x & 0x0f0f0f0fu,
                        __builtin_amdgcn_perm(QM.y, QM.x, 0x07050301u), __builtin_amdgcn_perm(QN.y, QN.x, 0x07050301u),
                        sc, code[1], qo[1]);
            duplex_word((SA.y >> 4) & 0x0f0f0f0fu, (SB.y >> 4) & 0x0f0f0f0fu,
                        __builtin_amdgcn_perm(QM.w, QM.z, 0x06040200u), __builtin_amdgcn_perm(QN.w, QN.z, 0x06040200u),
                        sc, code[2], qo[2]);
            duplex_word(SA.y & 0x0f0f0f0fu, SB.y & 0x0f0f0f0fu,
                        __builtin_amdgcn_perm(QM.w, QM.z, 0x07050301u), __builtin_amdgcn_perm(QN.w, QN.z, 0x07050301u),
                        sc, code[3], qo[3]);
            const uint32_t lm0 = __builtin_amdgcn_perm(lp[1], lp[0], 0x06040200u);
            const uint32_t lm1 = __builtin_amdgcn_perm(lp[1], lp[0], 0x07050301u);
            const uint32_t lm2 = __builtin_amdgcn_perm(lp[3], lp[2], 0x06040200u);
            const uint32_t lm3 = __builtin_amdgcn_perm(lp[3], lp[2], 0x07050301u);
            code[0] &= lm0; code[1] &= lm1; code[2] &= lm2; code[3] &= lm3;
            uint4 qout;
            qout.x = __builtin_amdgcn_perm(qo[1], qo[0], 0x05010400u) & lp[0];
            qout.y = __builtin_amdgcn_perm(qo[1], qo[0], 0x07030602u) & lp[1];
            qout.z = __builtin_amdgcn_perm(qo[3], qo[2], 0x05010400u) & lp[2];
            qout.w = __builtin_amdgcn_perm(qo[3], qo[2], 0x07030602u) & lp[3];
            *reinterpret_cast<uint4*>(out_qual + w * (int64_t)qstride + i0) = qout;
            *reinterpret_cast<uint2*>(out_seq + w * (int64_t)(qstride >> 1) + (i0 >> 1)) =
                make_uint2((code[0] << 4) | code[1], (code[2] << 4) | code[3]);
        }
        if (c == 0) {
            const int fa = (int)(ma.w & 0xfffu), fb = (int)(mb.w & 0xfffu);
            int32_t mapq = (int32_t)((ma.w >> 12) & 0xffu), tlen = (int32_t)ma.y, flag = fa, rg;
            const int32_t ra = TA.rg[a], rb = TBx.rg[b];
            if (sc) {
                rg = ra;
                if ((ma.w >> 20) & CC_RF_RG_UNSUPPORTED) eb |= EB_RG;
            } else {
                // read_mode over two reads: equal -> that value, else the first (tie, randint -> 0)
                if (fa == fb) flag = fa;
                else if (fa == 99 || fb == 99) flag = 99;
                else if (fa == 83 || fb == 83) flag = 83;
                else if (fa == 147 || fb == 147) flag = 147;
                else if (fa == 163 || fb == 163) flag = 163;
                rg = (ra >= 0 && rb >= 0) ? ra : -1;
                if (((ma.w | mb.w) >> 20) & CC_RF_RG_UNSUPPORTED) eb |= EB_RG;
            }
            out_meta[5 * w + 0] = L;
            out_meta[5 * w + 1] = mapq;
            out_meta[5 * w + 2] = tlen;
            out_meta[5 * w + 3] = flag;
            out_meta[5 * w + 4] = rg;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) eb |= __shfl_xor(eb, o);
    if (lane == 0 && eb) atomicOr(err, eb);
}

__global__ __launch_bounds__(256) void k_ckey_out(int64_t n, const int32_t* __restrict__ pairs, PairView V,
                                                  DevTable T, int32_t* __restrict__ out9) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t p = pairs[i];
    int32_t* o = out9 + 9 * i;
    if (p < 0) {
        for (int k = 0; k < 9; ++k) o[k] = -1;
        return;
    }
    const CKey c = ckey_of_pair(T, V, p);
    o[0] = c.bc; o[1] = c.tidLo; o[2] = c.posLo; o[3] = c.tidHi; o[4] = c.posHi;
    o[5] = c.cigA; o[6] = c.cigB; o[7] = (int32_t)(c.strand & 3u); o[8] = (int32_t)c.abstlen;
}

__global__ __launch_bounds__(256) void k_q_pairs(int64_t Q, const int32_t* __restrict__ ent_pair,
                                                 int32_t* __restrict__ out) {
    int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < Q) out[q] = ent_pair[q >> 1];
}


// ------------------------------------------------------------------ scans
// Reduce-then-scan over u32 flags (sum, exclusive) or group starts (max, inclusive):
// 4096-element tiles staged through LDS so every global access is a coalesced 16-B
// lane load/store; 12 B of HBM traffic per element (read, read, write) plus a tiny
// pass over the per-tile partials, which also leaves the total on the device.
constexpr int SCAN_T = 256, SCAN_I = 16, SCAN_TILE = SCAN_T * SCAN_I;

template <bool MAX>
__device__ __forceinline__ uint32_t sop(uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : a + b; }

// tile -> s_tile (coalesced), returns this thread's 16 contiguous elements
__device__ __forceinline__ void scan_load_tile(const uint32_t* __restrict__ in, int64_t n, int64_t base,
                                               uint32_t* s_tile, uint32_t v[SCAN_I]) {
    const int tid = threadIdx.x;
    if (base + SCAN_TILE <= n) {
#pragma unroll
        for (int j = 0; j < SCAN_I / 4; ++j) {
            const int o = (j * SCAN_T + tid) * 4;
            reinterpret_cast<uint4*>(s_tile)[o >> 2] = *reinterpret_cast<const uint4*>(in + base + o);
        }
    } else {
        for (int o = tid; o < SCAN_TILE; o += SCAN_T) s_tile[o] = base + o < n ? in[base + o] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SCAN_I / 4; ++j) {
        // rotate the 16-B reads by lane so a wave's ds_read_b128 spread over the banks
        const int jj = (j + (tid >> 1)) & 3;
        const uint4 q = reinterpret_cast<const uint4*>(s_tile)[tid * 4 + jj];
        v[4 * jj + 0] = q.x; v[4 * jj + 1] = q.y; v[4 * jj + 2] = q.z; v[4 * jj + 3] = q.w;
    }
}

template <bool MAX>
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t x, uint32_t* s_w, uint32_t* tot) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc = sop<MAX>(inc, y);
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t pre = 0, all = 0;
#pragma unroll
    for (int j = 0; j < SCAN_T / 64; ++j) {
        if (j < w) pre = sop<MAX>(pre, s_w[j]);
        all = sop<MAX>(all, s_w[j]);
    }
    *tot = all;
    uint32_t ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = 0;
    return sop<MAX>(pre, ex);
}

// the sum of the 4 byte flags (0/1) of a word
__device__ __forceinline__ uint32_t byte_sum(uint32_t w) { return (w * 0x01010101u) >> 24; }

template <bool MAX, class TIn>
__global__ __launch_bounds__(SCAN_T) void k_scan_reduce(const TIn* __restrict__ in, int64_t n,
                                                        uint32_t* __restrict__ part) {
    __shared__ uint32_t s_w[SCAN_T / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    const int tid = threadIdx.x;
    uint32_t acc = 0;
    if constexpr (sizeof(TIn) == 1) {
        static_assert(!MAX, "byte flags are summed");
        // one 16-B load per thread (SCAN_I byte flags)
        if (base + SCAN_TILE <= n) {
            const uint4 q = *reinterpret_cast<const uint4*>(in + base + tid * SCAN_I);
            acc = byte_sum(q.x) + byte_sum(q.y) + byte_sum(q.z) + byte_sum(q.w);
        } else {
            for (int o = tid; o < SCAN_TILE; o += SCAN_T)
                if (base + o < n) acc += in[base + o];
        }
    } else if (base + SCAN_TILE <= n) {
#pragma unroll
        for (int j = 0; j < SCAN_I / 4; ++j) {
            const uint4 q = *reinterpret_cast<const uint4*>(in + base + (j * SCAN_T + tid) * 4);
            acc = sop<MAX>(acc, sop<MAX>(sop<MAX>(q.x, q.y), sop<MAX>(q.z, q.w)));
        }
    } else {
        for (int o = tid; o < SCAN_TILE; o += SCAN_T)
            if (base + o < n) acc = sop<MAX>(acc, in[base + o]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc = sop<MAX>(acc, __shfl_xor(acc, o, 64));
    if ((tid & 63) == 0) s_w[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int j = 0; j < SCAN_T / 64; ++j) t = sop<MAX>(t, s_w[j]);
        part[blockIdx.x] = t;
    }
}

// out = exclusive prefix sum (MAX = false) or inclusive running max (MAX = true)
// Scan outputs.  ScanStore writes the prefix array; the Emit* consumers take (i, prefix, value)
// per element in the store phase instead, so a compaction needs neither the prefix array nor a
// pass of its own.
template <class E, class = void>
struct is_staged { static constexpr bool value = false; };
template <class E>
struct is_staged<E, std::void_t<decltype(E::kStaged)>> { static constexpr bool value = E::kStaged; };
struct ScanStore {
    static constexpr bool kPlain = true;
    uint32_t* out;
    __device__ void operator()(int64_t, uint32_t, uint32_t) const {}
};
// Staged emitters (kStaged) split an element's work into ld1 (loads indexed by the element), ld2
// (loads indexed by what ld1 read) and st (the stores), so the scan's store phase issues the loads
// of all of a thread's elements before waiting on any of them (k_scan_down).
struct EmitPairs {   // completed pairs (mate_of >= 0) in stream order of their second end: the two
                     // records, the completing region, and on a sorted table each record's read end
    static constexpr bool kPlain = false, kStaged = true;
    const int32_t* mate_of;
    int ident;
    const int32_t *stream_rec, *stream_region;
    int32_t *rec1, *rec2, *region, *rec_e;
    struct Ld { int32_t a, b, reg; };
    __device__ Ld ld1(int64_t i, uint32_t f) const {
        Ld l{-1, -1, 0};
        if (!f) return l;
        l.a = mate_of[i];
        l.b = ident ? (int32_t)i : stream_rec[i];
        l.reg = stream_region[i];
        return l;
    }
    __device__ void ld2(Ld& l, uint32_t f) const {
        if (f && !ident) l.a = stream_rec[l.a];
    }
    __device__ void st(int64_t, uint32_t x, uint32_t f, const Ld& l) const {
        if (!f) return;
        rec1[x] = l.a;
        rec2[x] = l.b;
        region[x] = l.reg < 0 ? -l.reg - 1 : l.reg;
        if (rec_e) { rec_e[l.a] = (int32_t)(2 * x); rec_e[l.b] = (int32_t)(2 * x + 1); }
    }
    __device__ void operator()(int64_t i, uint32_t x, uint32_t f) const {
        Ld l = ld1(i, f);
        ld2(l, f);
        st(i, x, f, l);
    }
};
struct EmitFamStarts {   // each family's first slot, and per family the members dropped ("line read twice")
    static constexpr bool kPlain = false;
    const uint32_t* validf;
    int32_t *fam_beg, *fam_drop;
    uint32_t* n_drop;
    int64_t cap;        // a planned re-run's family count: more families re-run the pass (EB_PLAN)
    uint32_t* err;
    __device__ void operator()(int64_t i, uint32_t x, uint32_t f) const {
        if ((int64_t)x >= cap + (f ? 0 : 1)) { atomicOr(err, EB_PLAN); return; }
        if (f) fam_beg[x] = (int32_t)i;
        else if (!validf[i]) { atomicAdd(&fam_drop[x - 1], 1); atomicAdd(n_drop, 1u); }   // rare
    }
};
struct EmitCreation {   // family creation order (tag_dict insertion order), each creation's pair and
                        // the family sizes in that order (read_families.txt, SSCS_maker.py:401-408)
    static constexpr bool kPlain = false, kStaged = true;
    const int32_t *cfam, *fam_n;
    int32_t *fam_by_k, *fam_k, *pair_by_k, *fsz;
    struct Ld { int32_t fm, n; };
    __device__ Ld ld1(int64_t i, uint32_t f) const { return Ld{f ? cfam[i] : -1, 0}; }
    __device__ void ld2(Ld& l, uint32_t f) const {
        if (f) l.n = fam_n[l.fm];
    }
    __device__ void st(int64_t i, uint32_t x, uint32_t f, const Ld& l) const {
        if (!f) return;
        fam_by_k[x] = l.fm;
        fam_k[l.fm] = (int32_t)x;
        pair_by_k[x] = (int32_t)(i >> 1);   // i is the creating read end (fam_first)
        fsz[x] = l.n;
    }
    __device__ void operator()(int64_t i, uint32_t x, uint32_t f) const {
        Ld l = ld1(i, f);
        ld2(l, f);
        st(i, x, f, l);
    }
};
struct EmitGather {   // out[x] = src[i] for the flagged i
    static constexpr bool kPlain = false;
    const int32_t* src;
    int32_t* out;
    __device__ void operator()(int64_t i, uint32_t x, uint32_t f) const {
        if (f) out[x] = src[i];
    }
};
struct EmitVotePairs {   // the duplex votes' pairs {read1, read2, decision, entry} by vote slot, and each
                         // entry's vote slot (-1: none)
    static constexpr bool kPlain = false, kStaged = true;
    const int32_t *t_rec, *p_rec, *dec;
    int32_t* vslot;
    int4* vpair;
    struct Ld { int32_t t, p, d; };
    __device__ Ld ld1(int64_t i, uint32_t f) const { return f ? Ld{t_rec[i], p_rec[i], dec[i]} : Ld{0, 0, 0}; }
    __device__ void ld2(Ld&, uint32_t) const {}
    __device__ void st(int64_t i, uint32_t x, uint32_t f, const Ld& l) const {
        vslot[i] = f ? (int32_t)x : -1;
        if (f) vpair[x] = make_int4(l.t, l.p, l.d, (int32_t)i);
    }
    __device__ void operator()(int64_t i, uint32_t x, uint32_t f) const {
        Ld l = ld1(i, f);
        st(i, x, f, l);
    }
};
struct EmitList {   // vote list of the flagged pairs and each pair's vote slot (-1: none)
    static constexpr bool kPlain = false;
    int32_t *vslot, *list;
    __device__ void operator()(int64_t i, uint32_t x, uint32_t f) const {
        vslot[i] = f ? (int32_t)x : -1;
        if (f) list[x] = (int32_t)i;
    }
};
struct EmitEntries {   // csn_pair_dict entries in creation order: the family pair and its read pair, and
                       // whether the entry has two tags (the SSCS region loop emits those: has2)
    static constexpr bool kPlain = false, kStaged = true;
    const int32_t *e1k, *fam_by_k, *pair_by_k;
    int32_t *ent_f, *ent_pair, *fam_o;
    uint8_t* has2;
    struct Ld { int32_t f0, k1, pr; };   // k1 becomes f1 in ld2
    __device__ Ld ld1(int64_t k, uint32_t f) const {
        return f ? Ld{fam_by_k[k], e1k[k], pair_by_k[k]} : Ld{-1, -1, -1};
    }
    __device__ void ld2(Ld& l, uint32_t f) const { l.k1 = f && l.k1 >= 0 ? fam_by_k[l.k1] : -1; }
    __device__ void st(int64_t, uint32_t r, uint32_t f, const Ld& l) const {
        if (!f) return;
        const int32_t f0 = l.f0, f1 = l.k1;
        ent_f[2 * r] = f0;
        ent_f[2 * r + 1] = f1;
        has2[r] = f1 >= 0 ? 1 : 0;
        ent_pair[r] = l.pr;
        fam_o[f0] = (int32_t)(2 * r);
        if (f1 >= 0) fam_o[f1] = (int32_t)(2 * r + 1);
    }
    __device__ void operator()(int64_t k, uint32_t r, uint32_t f) const {
        Ld l = ld1(k, f);
        ld2(l, f);
        st(k, r, f, l);
    }
};

// The tile's carry-in is the reduction of the partials of the tiles before it (L2-resident, a
// few KB), so no separate pass scans the partials; the last tile writes the total.
template <bool MAX, class Emit, class TIn>
__global__ __launch_bounds__(SCAN_T) void k_scan_down(const TIn* __restrict__ in, int64_t n,
                                                      const uint32_t* __restrict__ part,
                                                      uint32_t* __restrict__ total, Emit em) {
    __shared__ uint32_t s_tile[SCAN_TILE];
    __shared__ uint32_t s_w[SCAN_T / 64];
    __shared__ uint32_t s_pre[SCAN_T / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    const int tid = threadIdx.x;
    uint32_t pre = 0;
    for (uint32_t i = tid; i < blockIdx.x; i += SCAN_T) pre = sop<MAX>(pre, part[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pre = sop<MAX>(pre, __shfl_xor(pre, o, 64));
    if ((tid & 63) == 0) s_pre[tid >> 6] = pre;
    uint32_t v[SCAN_I];
    if constexpr (sizeof(TIn) == 1) {
        // the thread's 16 byte flags in one 16-B load (its elements are contiguous)
        if (base + SCAN_TILE <= n) {
            const uint4 q = *reinterpret_cast<const uint4*>(in + base + tid * SCAN_I);
            const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int k = 0; k < SCAN_I; ++k) v[k] = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
        } else {
#pragma unroll
            for (int k = 0; k < SCAN_I; ++k) {
                const int64_t i = base + tid * SCAN_I + k;
                v[k] = i < n ? (uint32_t)in[i] : 0u;
            }
        }
        __syncthreads();   // publishes s_pre
    } else {
        scan_load_tile(in, n, base, s_tile, v);   // its barrier publishes s_pre too
    }
    pre = 0;
#pragma unroll
    for (int j = 0; j < SCAN_T / 64; ++j) pre = sop<MAX>(pre, s_pre[j]);
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) t = sop<MAX>(t, v[k]);
    uint32_t all;
    uint32_t run = sop<MAX>(pre, block_scan_excl<MAX>(t, s_w, &all));
    if (blockIdx.x == gridDim.x - 1 && tid == 0) *total = sop<MAX>(pre, all);
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
        const uint32_t x = v[k];
        if (MAX) { run = sop<MAX>(run, x); v[k] = run; }
        else { v[k] = run; run += x; }
    }
#pragma unroll
    for (int j = 0; j < SCAN_I / 4; ++j) {
        const int jj = (j + (tid >> 1)) & 3;
        reinterpret_cast<uint4*>(s_tile)[tid * 4 + jj] = make_uint4(v[4 * jj], v[4 * jj + 1], v[4 * jj + 2], v[4 * jj + 3]);
    }
    __syncthreads();
    if (base + SCAN_TILE <= n) {
#pragma unroll
        for (int j = 0; j < SCAN_I / 4; ++j) {
            const int o = (j * SCAN_T + tid) * 4;
            const uint4 x = reinterpret_cast<const uint4*>(s_tile)[o >> 2];
            if constexpr (Emit::kPlain) {
                *reinterpret_cast<uint4*>(em.out + base + o) = x;
            } else if constexpr (sizeof(TIn) == 1 && is_staged<Emit>::value) {
                continue;   // (below: all of the thread's elements at once)
            } else if constexpr (sizeof(TIn) == 1) {
                const uint32_t f = *reinterpret_cast<const uint32_t*>(in + base + o);   // L2-resident
                em(base + o, x.x, f & 0xffu);
                em(base + o + 1, x.y, (f >> 8) & 0xffu);
                em(base + o + 2, x.z, (f >> 16) & 0xffu);
                em(base + o + 3, x.w, f >> 24);
            } else {
                const uint4 f = *reinterpret_cast<const uint4*>(in + base + o);   // L2-resident
                em(base + o, x.x, f.x);
                em(base + o + 1, x.y, f.y);
                em(base + o + 2, x.z, f.z);
                em(base + o + 3, x.w, f.w);
            }
        }
        if constexpr (!Emit::kPlain && sizeof(TIn) == 1 && is_staged<Emit>::value) {
            // the thread's 16 elements: every ld1, then every ld2, then the stores
            typename Emit::Ld ld[SCAN_I];
            uint32_t fx[SCAN_I], xx[SCAN_I];
#pragma unroll
            for (int j = 0; j < SCAN_I / 4; ++j) {
                const int o = (j * SCAN_T + tid) * 4;
                const uint4 x = reinterpret_cast<const uint4*>(s_tile)[o >> 2];
                const uint32_t f = *reinterpret_cast<const uint32_t*>(in + base + o);   // L2-resident
                xx[4 * j] = x.x; xx[4 * j + 1] = x.y; xx[4 * j + 2] = x.z; xx[4 * j + 3] = x.w;
#pragma unroll
                for (int k = 0; k < 4; ++k) fx[4 * j + k] = (f >> (8 * k)) & 0xffu;
            }
#pragma unroll
            for (int e = 0; e < SCAN_I; ++e) ld[e] = em.ld1(base + ((e >> 2) * SCAN_T + tid) * 4 + (e & 3), fx[e]);
#pragma unroll
            for (int e = 0; e < SCAN_I; ++e) em.ld2(ld[e], fx[e]);
#pragma unroll
            for (int e = 0; e < SCAN_I; ++e) em.st(base + ((e >> 2) * SCAN_T + tid) * 4 + (e & 3), xx[e], fx[e], ld[e]);
        }
    } else {
        for (int o = tid; o < SCAN_TILE; o += SCAN_T) {
            if (base + o >= n) continue;
            if constexpr (Emit::kPlain) em.out[base + o] = s_tile[o];
            else em(base + o, s_tile[o], (uint32_t)in[base + o]);
        }
    }
}

// The same scan in one launch (decoupled look-back): each block draws its tile in launch order from
// a ticket (so every tile it waits on belongs to a block already running), publishes its tile's
// aggregate, then wave 0 walks back over the published states 64 tiles at a time, adding aggregates
// until it meets a tile whose inclusive prefix is known, and publishes its own inclusive prefix.
// A state word is epoch (30 b) | kind (2 b: 1 aggregate, 2 inclusive prefix) | value (32 b); the
// launch's epoch makes the words of earlier launches read as "not yet published", so the state
// array is never cleared.  The last ticket resets the ticket counter for the next launch.
struct ScanLB {
    unsigned long long* st;   // per tile state
    uint32_t* ticket;
    uint32_t epoch;           // 1 .. 2^30 - 1
    uint32_t* err;
};
constexpr uint32_t SCAN_SPIN_MAX = 1u << 22;   // look-back polls of one state before EB_SCANWAIT
__device__ __forceinline__ void lb_publish(const ScanLB& lb, uint32_t tile, uint32_t kind, uint32_t v) {
    __hip_atomic_store(lb.st + tile, ((unsigned long long)lb.epoch << 34) | ((unsigned long long)kind << 32) | v,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool MAX, class Emit, class TIn>
__global__ __launch_bounds__(SCAN_T) void k_scan_one(const TIn* __restrict__ in, int64_t n, int64_t nb,
                                                     uint32_t* __restrict__ total, Emit em, ScanLB lb) {
    __shared__ uint32_t s_tile[SCAN_TILE];
    __shared__ uint32_t s_w[SCAN_T / 64];
    __shared__ uint32_t s_id[2];   // [0] the tile, [1] its exclusive prefix
    const int tid = threadIdx.x;
    if (tid == 0) {
        const uint32_t b = atomicAdd(lb.ticket, 1u);
        if ((int64_t)b == nb - 1) atomicExch(lb.ticket, 0u);   // every ticket is drawn
        s_id[0] = b;
    }
    __syncthreads();
    const uint32_t b = s_id[0];
    const int64_t base = (int64_t)b * SCAN_TILE;
    uint32_t v[SCAN_I];
    if constexpr (sizeof(TIn) == 1) {
        if (base + SCAN_TILE <= n) {
            const uint4 q = *reinterpret_cast<const uint4*>(in + base + tid * SCAN_I);
            const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int k = 0; k < SCAN_I; ++k) v[k] = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
        } else {
#pragma unroll
            for (int k = 0; k < SCAN_I; ++k) {
                const int64_t i = base + tid * SCAN_I + k;
                v[k] = i < n ? (uint32_t)in[i] : 0u;
            }
        }
    } else {
        scan_load_tile(in, n, base, s_tile, v);
    }
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) t = sop<MAX>(t, v[k]);
    uint32_t all;
    uint32_t run = block_scan_excl<MAX>(t, s_w, &all);
    if (tid < 64) {
        uint32_t excl = 0;
        if (b == 0) {
            if (tid == 0) lb_publish(lb, 0, 2u, all);
        } else {
            if (tid == 0) lb_publish(lb, b, 1u, all);
            int64_t j = (int64_t)b - 1;
            bool late = false;
            for (;;) {
                const int64_t i = j - tid;   // lane 0: the nearest tile
                uint32_t kind = 2u, val = 0u;
                if (i >= 0) {
                    unsigned long long sv = 0;
                    for (uint32_t spin = 0;; ++spin) {
                        sv = __hip_atomic_load(lb.st + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((uint32_t)(sv >> 34) == lb.epoch && ((sv >> 32) & 3u) != 0u) break;
                        if (spin >= SCAN_SPIN_MAX) { late = true; sv = 2ULL << 32; break; }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    kind = (uint32_t)(sv >> 32) & 3u;
                    val = (uint32_t)sv;
                }
                const uint64_t im = __ballot(kind == 2u);
                const int first = im ? __ffsll((unsigned long long)im) - 1 : 64;
                uint32_t x = tid <= first ? val : 0u;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) x = sop<MAX>(x, __shfl_xor(x, o, 64));
                excl = sop<MAX>(excl, x);
                if (im) break;
                j -= 64;
            }
            if (tid == 0) {
                lb_publish(lb, b, 2u, sop<MAX>(excl, all));
                if (late) atomicOr(lb.err, EB_SCANWAIT);
            }
        }
        if (tid == 0) s_id[1] = excl;
    }
    __syncthreads();
    const uint32_t pre = s_id[1];
    run = sop<MAX>(pre, run);
    if ((int64_t)b == nb - 1 && tid == 0) *total = sop<MAX>(pre, all);
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
        const uint32_t x = v[k];
        if (MAX) { run = sop<MAX>(run, x); v[k] = run; }
        else { v[k] = run; run += x; }
    }
#pragma unroll
    for (int j = 0; j < SCAN_I / 4; ++j) {
        const int jj = (j + (tid >> 1)) & 3;
        reinterpret_cast<uint4*>(s_tile)[tid * 4 + jj] = make_uint4(v[4 * jj], v[4 * jj + 1], v[4 * jj + 2], v[4 * jj + 3]);
    }
    __syncthreads();
    if (base + SCAN_TILE <= n) {
#pragma unroll
        for (int j = 0; j < SCAN_I / 4; ++j) {
            const int o = (j * SCAN_T + tid) * 4;
            const uint4 x = reinterpret_cast<const uint4*>(s_tile)[o >> 2];
            if constexpr (Emit::kPlain) {
                *reinterpret_cast<uint4*>(em.out + base + o) = x;
            } else if constexpr (sizeof(TIn) == 1 && is_staged<Emit>::value) {
                continue;   // (below: all of the thread's elements at once)
            } else if constexpr (sizeof(TIn) == 1) {
                const uint32_t f = *reinterpret_cast<const uint32_t*>(in + base + o);   // L2-resident
                em(base + o, x.x, f & 0xffu);
                em(base + o + 1, x.y, (f >> 8) & 0xffu);
                em(base + o + 2, x.z, (f >> 16) & 0xffu);
                em(base + o + 3, x.w, f >> 24);
            } else {
                const uint4 f = *reinterpret_cast<const uint4*>(in + base + o);   // L2-resident
                em(base + o, x.x, f.x);
                em(base + o + 1, x.y, f.y);
                em(base + o + 2, x.z, f.z);
                em(base + o + 3, x.w, f.w);
            }
        }
        if constexpr (!Emit::kPlain && sizeof(TIn) == 1 && is_staged<Emit>::value) {
            // the thread's 16 elements: every ld1, then every ld2, then the stores
            typename Emit::Ld ld[SCAN_I];
            uint32_t fx[SCAN_I], xx[SCAN_I];
#pragma unroll
            for (int j = 0; j < SCAN_I / 4; ++j) {
                const int o = (j * SCAN_T + tid) * 4;
                const uint4 x = reinterpret_cast<const uint4*>(s_tile)[o >> 2];
                const uint32_t f = *reinterpret_cast<const uint32_t*>(in + base + o);   // L2-resident
                xx[4 * j] = x.x; xx[4 * j + 1] = x.y; xx[4 * j + 2] = x.z; xx[4 * j + 3] = x.w;
#pragma unroll
                for (int k = 0; k < 4; ++k) fx[4 * j + k] = (f >> (8 * k)) & 0xffu;
            }
#pragma unroll
            for (int e = 0; e < SCAN_I; ++e) ld[e] = em.ld1(base + ((e >> 2) * SCAN_T + tid) * 4 + (e & 3), fx[e]);
#pragma unroll
            for (int e = 0; e < SCAN_I; ++e) em.ld2(ld[e], fx[e]);
#pragma unroll
            for (int e = 0; e < SCAN_I; ++e) em.st(base + ((e >> 2) * SCAN_T + tid) * 4 + (e & 3), xx[e], fx[e], ld[e]);
        }
    } else {
        for (int o = tid; o < SCAN_TILE; o += SCAN_T) {
            if (base + o >= n) continue;
            if constexpr (Emit::kPlain) em.out[base + o] = s_tile[o];
            else em(base + o, s_tile[o], (uint32_t)in[base + o]);
        }
    }
}

// A deferred pass's readback in one launch instead of three copies: the error word, the counters
// summed over their stripes and the planned totals, written straight into the pass's slot of the
// pinned (device-visible) readback area: h + 0 error word, h + 256 totals, h + 1024 counters.
// a plan slot's striped count (stripe_add) not folded by k_stripe_total during the pass
__device__ __forceinline__ uint32_t stripe_sum(const uint32_t* __restrict__ stripes, int slot) {
    uint32_t v = 0;
    if (stripes)
        for (int k = 0; k < PSTRIPES; ++k) v += stripes[((int64_t)slot * PSTRIPES + k) * PSTRIDE];
    return v;
}

__global__ __launch_bounds__(256) void k_defer_pack(const uint32_t* __restrict__ err,
                                                    const unsigned long long* __restrict__ cnt,
                                                    const uint32_t* __restrict__ plan, int nplan,
                                                    const uint32_t* __restrict__ stripes, uint8_t* __restrict__ h) {
    const int t = threadIdx.x;
    if (t == 0) *reinterpret_cast<uint32_t*>(h) = *err;
    if (cnt && t < CC_NUM_COUNTERS) {
        unsigned long long v = 0;
        for (int k = 0; k < CNT_STRIPES; ++k) v += cnt[CC_NUM_COUNTERS * k + t];
        reinterpret_cast<unsigned long long*>(h + 1024)[t] = v;
    }
    if (plan)
        for (int i = t; i < nplan; i += blockDim.x)
            reinterpret_cast<uint32_t*>(h + 256)[i] = plan[i] + stripe_sum(stripes, i);
}

// the same fold into the plan slots themselves (a planned pass read back without deferral)
__global__ __launch_bounds__(64) void k_stripe_fold(const uint32_t* __restrict__ stripes, uint32_t* __restrict__ plan,
                                                    int nplan) {
    for (int i = threadIdx.x; i < nplan; i += blockDim.x) plan[i] += stripe_sum(stripes, i);
}

// ================================================================== host side
namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    size_t used = 0;
};

struct Group {
    int32_t table = -1;
    int64_t S = 0, P = 0, R = 0, F = 0, E = 0, Q = 0, NV = 0;
    uint64_t seed = 0;
    int scoped = 0, delim_filter = 0, badread = 0;
    uint64_t ht_mask = 0;
    bool csn_fast = false;
    bool stripes_pending = false;   // striped plan counts left for the end-of-pass fold
    bool no_deep_fam = false;       // deep groups ranked by the sort (a long family out of end order)
    int coord_sorted = 0;
    bool force_sort = false;     // pair by the qname sort even on a sorted table (qnames seen 3+ times)
    int ident = 0;               // stream_rec[s] == s for every s (the whole table in file order)
    bool local_groups = false;   // families of each position group contiguous (coordinate grouping, no deep group)
    int64_t counters[CC_NUM_COUNTERS] = {0};
    std::map<std::string, DevBuf> buf;
    // Launch plan: every device-side total (scan totals, the csn sharing flag) of the last exact
    // pass of each stage on this group, keyed by name.  A re-run on the same resident stream takes
    // its sizes and grids from the plan instead of waiting for each total, and checks all of them
    // against the device in the one readback at the end; a mismatch re-runs the stage exactly.
    std::map<std::string, int64_t> plan;
    std::map<std::string, int> slot;
    std::map<std::string, bool> planned;   // stage -> has a complete plan
    bool fast = false;
    bool members_built = false;  // mem_meta holds the last pass's member records
    int64_t n_deepg = 0;         // deep position groups of the last pass (k_build_meta's list)
    bool fam_tags_built = false; // fam_tag holds the last pass's family tags
    bool overlap = false;        // the stream holds a record twice (overlapping bed regions)
    std::vector<std::string> verify;
    std::vector<int32_t> swap_host;   // the barcode swap table last uploaded (bc_swap)
    double thr_cutoff = -1.0;         // the cutoff cutoff_thr holds (k_cutoff_table, once per cutoff)
};

// A planned pass's end-of-pass check while the context defers them (cc_defer): its readback was
// enqueued into a slot of the deferred pinned area and is judged by cc_commit.
struct DeferredCheck {
    Group* g = nullptr;
    int32_t gid = -1;
    int slot = 0;
    bool counters = false;
    bool bad_listed = false;                        // g's BAD_LISTED > 0 when the pass ran
    std::vector<std::pair<int, int64_t>> expect;    // plan slot -> planned total
};
constexpr int DEFER_SLOTS = 64;
constexpr size_t DEFER_SLOT_BYTES = 12288;   // err word, plan totals at 256, counters at 1024

constexpr int CC_E_PLAN = -100;   // internal: a planned total did not hold (re-run exactly)
constexpr int CC_E_NEEDSORT = -101;   // internal: coordinate pairing met a qname seen 3+ times
constexpr int CC_E_DEEPSORT = -102;   // internal: a deep family needs the sorted deep-group path
constexpr int PLAN_SLOTS = 64;

}  // namespace

struct cc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    std::map<int32_t, DevTable> tables;
    std::map<int32_t, std::vector<void*>> table_allocs;
    std::map<int32_t, std::unique_ptr<Group>> groups;
    int32_t next_id = 1;
    DevBuf tmp;                     // rocprim temporary storage
    unsigned long long* scan_st = nullptr;   // k_scan_one's tile states (zeroed when allocated)
    uint32_t* scan_ticket = nullptr;
    int64_t scan_cap = 0;
    uint32_t scan_epoch = 0;
    uint32_t* d_err = nullptr;      // device error word
    unsigned long long* d_cnt = nullptr;
    void* h_pinned = nullptr;       // small pinned scratch for scalar readbacks
    bool profiling = false;
    std::unordered_set<std::string> prof_only;   // when non-empty, the only scopes timed
    struct Prof { double ms = 0; int64_t n = 0; };
    std::map<std::string, Prof> prof;
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
    std::vector<hipEvent_t> event_pool;   // recycled timing events (no hipEventCreate per launch)
    std::unique_ptr<Group> scratch;       // buffers of the function-level calls (cc_sscs_vote, cc_pair_vote)
    bool defer = false;                   // planned passes enqueue their checks (cc_defer / cc_commit)
    std::vector<DeferredCheck> deferred;
    uint8_t* h_defer = nullptr;           // DEFER_SLOTS pinned readback slots
    uint8_t* d_defer = nullptr;           // the same area as the device sees it (k_defer_pack)
};

namespace {

#define HIPCHK(x)                                                                               \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            ctx->err = std::string("HIP error ") + hipGetErrorString(e_) + " at " #x;           \
            return CC_E_HIP;                                                                    \
        }                                                                                       \
    } while (0)

#define RC(x)                     \
    do {                          \
        int rc_ = (x);            \
        if (rc_) return rc_;      \
    } while (0)

inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

// fills gathered for one k_fill launch (flushed when full or by launch())
struct Fills {
    cc_ctx* ctx;
    FillSet fs{};
    int64_t maxw = 0;
    explicit Fills(cc_ctx* c) : ctx(c) { fs.k = 0; }
    int add(void* p, size_t bytes, uint32_t word) {
        if (!p || bytes < 4) return 0;
        if (fs.k == FillSet::K) { int rc = launch(); if (rc) return rc; }
        fs.p[fs.k] = (uint32_t*)p;
        fs.n[fs.k] = (int64_t)(bytes / 4);
        fs.v[fs.k] = word;
        maxw = std::max<int64_t>(maxw, (int64_t)(bytes / 4));
        ++fs.k;
        return 0;
    }
    int launch();
};

template <typename T>
T* gbuf(cc_ctx* ctx, Group& g, const char* name, int64_t count, int* rc) {
    DevBuf& b = g.buf[name];
    size_t need = (size_t)std::max<int64_t>(count, 1) * sizeof(T);
    if (b.bytes < need) {
        if (b.p) (void)hipFree(b.p);
        b.p = nullptr;
        hipError_t e = hipMalloc(&b.p, need);
        if (e != hipSuccess) {
            ctx->err = std::string("hipMalloc failed for ") + name + ": " + hipGetErrorString(e);
            *rc = CC_E_HIP;
            b.bytes = 0;
            return nullptr;
        }
        b.bytes = need;
    }
    b.used = (size_t)std::max<int64_t>(count, 0) * sizeof(T);
    return (T*)b.p;
}

void* tmp_storage(cc_ctx* ctx, size_t bytes, int* rc) {
    if (ctx->tmp.bytes < bytes) {
        if (ctx->tmp.p) (void)hipFree(ctx->tmp.p);
        ctx->tmp.p = nullptr;
        size_t nb = bytes + bytes / 4 + 4096;
        if (hipMalloc(&ctx->tmp.p, nb) != hipSuccess) {
            ctx->err = "hipMalloc temp storage failed";
            *rc = CC_E_HIP;
            ctx->tmp.bytes = 0;
            return nullptr;
        }
        ctx->tmp.bytes = nb;
    }
    return ctx->tmp.p;
}

struct ProfScope {
    cc_ctx* ctx;
    const char* name;
    hipEvent_t a = nullptr, b = nullptr;
    static hipEvent_t take(cc_ctx* ctx) {
        hipEvent_t e = nullptr;
        if (!ctx->event_pool.empty()) {
            e = ctx->event_pool.back();
            ctx->event_pool.pop_back();
        } else {
            (void)hipEventCreate(&e);
        }
        return e;
    }
    ProfScope(cc_ctx* c, const char* n) : ctx(c), name(n) {
        if (ctx->profiling && !ctx->prof_only.empty() && !ctx->prof_only.count(n)) name = nullptr;
        if (ctx->profiling && name) {
            a = take(ctx);
            b = take(ctx);
            (void)hipEventRecord(a, ctx->stream);
        }
    }
    ~ProfScope() {
        if (ctx->profiling && name) {
            (void)hipEventRecord(b, ctx->stream);
            ctx->pending.push_back({name, {a, b}});
        }
    }
};

void flush_prof(cc_ctx* ctx) {
    if (ctx->pending.empty()) return;
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& p : ctx->pending) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, p.second.first, p.second.second);
        auto& pr = ctx->prof[p.first];
        pr.ms += ms;
        pr.n += 1;
        ctx->event_pool.push_back(p.second.first);
        ctx->event_pool.push_back(p.second.second);
    }
    ctx->pending.clear();
}

int sort_pairs(cc_ctx* ctx, const uint64_t* kin, uint64_t* kout, const uint32_t* vin, uint32_t* vout, int64_t n,
               const char* name, unsigned begin_bit = 0, unsigned end_bit = 64) {
    if (n <= 0) return 0;
    size_t bytes = 0;
    HIPCHK(rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, vin, vout, (size_t)n, begin_bit, end_bit, ctx->stream));
    int rc = 0;
    void* t = tmp_storage(ctx, bytes, &rc);
    if (!t) return rc;
    ProfScope ps(ctx, name);
    g_launches.fetch_add(1, std::memory_order_relaxed);
    HIPCHK(rocprim::radix_sort_pairs(t, bytes, kin, kout, vin, vout, (size_t)n, begin_bit, end_bit, ctx->stream));
    return 0;
}

// One look-back launch (k_scan_one) for scans of at most SCAN_ONE_MAX tiles (one look-back window:
// the reduce launch is a fixed ~3 us on the C5 trace), the reduce-then-scan pair above that; CC_SCAN1
// = 1 / 0 forces one or the other.  The total lands in d_tot (device).  Measured with the single
// launch for every scan: C2 1.08 -> 1.37 ms of scans per step (the look-back chain over ~4,900 tiles
// of a 20 M-entry scan costs more than the second pass over L2-resident flags), C5 1.612 -> 1.596 ms
// (profiles/r04_scan1_*).
constexpr int64_t SCAN_ONE_MAX = 64;
template <bool MAX, class Emit, class TIn>
int scan_launch(cc_ctx* ctx, const TIn* in, int64_t n, uint32_t* d_tot, const char* name, Emit em) {
    const int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    uintptr_t al = (uintptr_t)in;
    if constexpr (Emit::kPlain) al |= (uintptr_t)em.out;
    if (al & 15u) { ctx->err = "scan operands must be 16-B aligned"; return CC_E_INVALID; }
    const char* force = getenv("CC_SCAN1");
    const bool one = force ? force[0] == '1' : nb <= SCAN_ONE_MAX;
    if (one && nb > 0) {
        if (nb > ctx->scan_cap) {
            const int64_t cap = std::max<int64_t>(nb, 1 << 14);
            if (ctx->scan_st) {
                HIPCHK(hipStreamSynchronize(ctx->stream));   // earlier scans may still read the states
                (void)hipFree(ctx->scan_st);
            }
            ctx->scan_st = nullptr;
            ctx->scan_cap = 0;
            HIPCHK(hipMalloc((void**)&ctx->scan_st, sizeof(unsigned long long) * cap + 64));
            HIPCHK(hipMemsetAsync(ctx->scan_st, 0, sizeof(unsigned long long) * cap + 64, ctx->stream));
            ctx->scan_ticket = reinterpret_cast<uint32_t*>(ctx->scan_st + cap);   // (zeroed with the states)
            ctx->scan_cap = cap;
            ctx->scan_epoch = 0;
        }
        if (++ctx->scan_epoch >= (1u << 30)) {   // epochs exhausted: clear the states and restart
            HIPCHK(hipMemsetAsync(ctx->scan_st, 0, sizeof(unsigned long long) * ctx->scan_cap, ctx->stream));
            ctx->scan_epoch = 1;
        }
        const ScanLB lb{ctx->scan_st, ctx->scan_ticket, ctx->scan_epoch, ctx->d_err};
        ProfScope ps(ctx, name);
        hipLaunchKernelGGL((k_scan_one<MAX, Emit, TIn>), dim3((unsigned)nb), dim3(SCAN_T), 0, ctx->stream, in, n, nb,
                           d_tot, em, lb);
        return 0;
    }
    int rc = 0;
    uint32_t* part = (uint32_t*)tmp_storage(ctx, (size_t)nb * 4 + 64, &rc);
    if (!part) return rc;
    ProfScope ps(ctx, name);
    hipLaunchKernelGGL((k_scan_reduce<MAX, TIn>), dim3((unsigned)nb), dim3(SCAN_T), 0, ctx->stream, in, n, part);
    hipLaunchKernelGGL((k_scan_down<MAX, Emit, TIn>), dim3((unsigned)nb), dim3(SCAN_T), 0, ctx->stream, in, n, part, d_tot, em);
    return 0;
}



// Waits for the engine's stream by polling it: the pass readbacks wait for short tails of work,
// and a blocking wait's wake-up costs tens of microseconds per pass.  The hot poll is bounded
// (200 us); a longer wait yields the core between polls (the host's BGZF threads, other ranks).
hipError_t stream_wait(cc_ctx* ctx) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; ++i) {
        const hipError_t e = hipStreamQuery(ctx->stream);
        if (e != hipErrorNotReady) return e;
        if ((i & 63u) == 63u && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) sched_yield();
    }
}

// the debug build's first failed bounds check (site, index), reported as CC_E_INVALID
int dbg_fault(cc_ctx* ctx) {
#ifdef CC_DEBUG_BOUNDS
    unsigned long long f = 0;
    HIPCHK(hipMemcpyFromSymbol(&f, HIP_SYMBOL(g_dbg_fault), sizeof(f), 0, hipMemcpyDeviceToHost));
    if (f) {
        const unsigned long long zero = 0;   // reported once
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_fault), &zero, sizeof(zero), 0, hipMemcpyHostToDevice));
        static const char* names[] = {"?", "record index", "qname offset", "payload offset", "ranked slot", "pair",
                                      "member record", "vote record"};
        const int site = (int)(f >> 48);
        char buf[160];
        snprintf(buf, sizeof buf, "device bounds check failed: %s %lld out of range (debug build)",
                 names[site >= 0 && site < 8 ? site : 0], (long long)(int64_t)(f & 0xffffffffffffULL));
        ctx->err = buf;
        return CC_E_INVALID;
    }
#else
    (void)ctx;
#endif
    return 0;
}

int Fills::launch() {
    if (fs.k == 0) return 0;
    const unsigned blocks = std::min<unsigned>(nblk((maxw + 3) / 4), 2048u);
    hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, ctx->stream, fs);
    fs.k = 0;
    maxw = 0;
    return hipGetLastError() == hipSuccess ? 0 : CC_E_HIP;
}

uint32_t* plan_slot(cc_ctx* ctx, Group& g, const char* name, int* rc) {
    uint32_t* dtot = gbuf<uint32_t>(ctx, g, "plan_totals", PLAN_SLOTS, rc);
    if (*rc) return nullptr;
    auto it = g.slot.find(name);
    const int s = it != g.slot.end() ? it->second : (int)g.slot.size();
    if (s >= PLAN_SLOTS) { ctx->err = "too many planned totals"; *rc = CC_E_INVALID; return nullptr; }
    g.slot[name] = s;
    return dtot + s;
}

// the stripes of a plan slot's count (stripe_add / k_stripe_total), zeroed once when created
uint32_t* plan_stripes(cc_ctx* ctx, Group& g, uint32_t* slot, int* rc) {
    const bool fresh = !g.buf.count("plan_stripes") || !g.buf["plan_stripes"].p;
    uint32_t* st = gbuf<uint32_t>(ctx, g, "plan_stripes", (int64_t)PLAN_SLOTS * PSTRIPES * PSTRIDE, rc);
    if (*rc) return nullptr;
    if (fresh && hipMemsetAsync(st, 0, sizeof(uint32_t) * PLAN_SLOTS * PSTRIPES * PSTRIDE, ctx->stream) != hipSuccess) {
        *rc = CC_E_HIP;
        return nullptr;
    }
    return st + (slot - (uint32_t*)g.buf["plan_totals"].p) * (int64_t)PSTRIPES * PSTRIDE;
}

// A device total: on a planned re-run the plan's value (checked at the end), otherwise read back
// now (synchronises) and recorded in the plan.
int planned_total(cc_ctx* ctx, Group& g, const char* name, uint32_t* d_tot, int64_t* total) {
    if (g.fast && g.plan.count(name)) {
        *total = g.plan[name];
        g.verify.push_back(name);
        return 0;
    }
    uint32_t* h = (uint32_t*)ctx->h_pinned;
    HIPCHK(hipMemcpyAsync(h, d_tot, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(stream_wait(ctx));
    *total = (int64_t)h[0];
    g.plan[name] = *total;
    return 0;
}

// exclusive scan of u32 or byte flags with a planned total
template <class TIn>
int scan_total(cc_ctx* ctx, Group& g, const TIn* in, uint32_t* out, int64_t n, int64_t* total,
               const char* name) {
    if (n <= 0) { *total = 0; return 0; }
    int rc = 0;
    uint32_t* d_tot = plan_slot(ctx, g, name, &rc);
    if (rc) return rc;
    RC(scan_launch<false>(ctx, in, n, d_tot, name, ScanStore{out}));
    return planned_total(ctx, g, name, d_tot, total);
}

// exclusive scan of u32 or byte flags consumed by an emitter (compaction in the scan's store phase)
template <class Emit, class TIn>
int scan_emit(cc_ctx* ctx, Group& g, const TIn* in, int64_t n, int64_t* total, const char* name, Emit em) {
    if (n <= 0) { *total = 0; return 0; }
    int rc = 0;
    uint32_t* d_tot = plan_slot(ctx, g, name, &rc);
    if (rc) return rc;
    RC(scan_launch<false>(ctx, in, n, d_tot, name, em));
    return planned_total(ctx, g, name, d_tot, total);
}

// End of a stage pass: ONE readback of the error word, the read_bam counters (optional) and the
// planned totals this pass relied on.  *plan_ok = false when one of them did not hold.
// A planned pass on a deferring context enqueues the same readback into a slot of its own and
// returns at once (cc_commit judges it); nothing here waits for the device then.
int finish_pass(cc_ctx* ctx, Group& g, uint32_t* bits, bool counters, bool* plan_ok) {
    if (ctx->defer && g.fast && ctx->h_defer && ctx->deferred.size() < (size_t)DEFER_SLOTS) {
        DeferredCheck d;
        d.g = &g;
        for (auto& kv : ctx->groups)
            if (kv.second.get() == &g) d.gid = kv.first;
        d.slot = (int)ctx->deferred.size();
        d.counters = counters;
        d.bad_listed = g.counters[CC_CNT_BAD_LISTED] > 0;
        uint8_t* dh = ctx->d_defer + (size_t)d.slot * DEFER_SLOT_BYTES;
        const bool totals = !g.verify.empty();
        hipLaunchKernelGGL(k_defer_pack, dim3(1), dim3(256), 0, ctx->stream, (const uint32_t*)ctx->d_err,
                           counters ? (const unsigned long long*)ctx->d_cnt : nullptr,
                           totals ? (const uint32_t*)g.buf["plan_totals"].p : nullptr, PLAN_SLOTS,
                           g.stripes_pending ? (const uint32_t*)g.buf["plan_stripes"].p : nullptr, dh);
        g.stripes_pending = false;
        if (totals)
            for (const auto& nm : g.verify) d.expect.push_back({g.slot[nm], g.plan[nm]});
        g.verify.clear();
        ctx->deferred.push_back(std::move(d));
        *bits = 0;
        *plan_ok = true;
        return 0;
    }
    uint8_t* h = (uint8_t*)ctx->h_pinned;
    HIPCHK(hipMemcpyAsync(h + 16, ctx->d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
    if (counters)
        HIPCHK(hipMemcpyAsync(h + 1024, ctx->d_cnt, sizeof(unsigned long long) * CC_NUM_COUNTERS * CNT_STRIPES,
                              hipMemcpyDeviceToHost,
                              ctx->stream));
    if (g.stripes_pending) {
        hipLaunchKernelGGL(k_stripe_fold, dim3(1), dim3(64), 0, ctx->stream, (const uint32_t*)g.buf["plan_stripes"].p,
                           (uint32_t*)g.buf["plan_totals"].p, PLAN_SLOTS);
        g.stripes_pending = false;
    }
    if (!g.verify.empty())
        HIPCHK(hipMemcpyAsync(h + 256, g.buf["plan_totals"].p, 4 * PLAN_SLOTS, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(stream_wait(ctx));
    RC(dbg_fault(ctx));
    *bits = *(uint32_t*)(h + 16);
    const bool cap_over = (*bits & EB_PLAN) != 0;
    *bits &= ~EB_PLAN;
    if (counters)
        for (int i = 0; i < CC_NUM_COUNTERS; ++i) {
            int64_t t = 0;
            for (int k = 0; k < CNT_STRIPES; ++k) t += (int64_t)((unsigned long long*)(h + 1024))[CC_NUM_COUNTERS * k + i];
            g.counters[i] = t;
        }
    *plan_ok = !cap_over;
    for (const auto& nm : g.verify)
        if ((int64_t)((uint32_t*)(h + 256))[g.slot[nm]] != g.plan[nm]) *plan_ok = false;
    g.verify.clear();
    return 0;
}

// Run a stage pass planned (when the group has a plan for it) and exactly otherwise or when the
// plan did not hold; the exact pass records the plan.
template <typename Pass>
int run_planned(cc_ctx* ctx, Group& g, const char* stage, Pass pass) {
    if (g.planned[stage]) {
        g.fast = true;
        g.verify.clear();
        const int rc = pass();
        g.fast = false;
        if (rc != CC_E_PLAN) return rc;
    }
    g.verify.clear();
    const int rc = pass();
    g.planned[stage] = rc == 0;
    return rc;
}

int read_err(cc_ctx* ctx, uint32_t* bits) {
    uint32_t* h = (uint32_t*)ctx->h_pinned + 4;
    HIPCHK(hipMemcpyAsync(h, ctx->d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(stream_wait(ctx));
    *bits = *h;
    return dbg_fault(ctx);
}

int err_code(cc_ctx* ctx, uint32_t bits) {
    if (!bits) return 0;
    if (bits & EB_COLLISION) { ctx->err = "64-bit key hash collision (retry with another seed)"; return CC_E_COLLISION; }
    if (bits & EB_KEYERROR) { ctx->err = "KeyError: read_dict[tag] already deleted (consensus_helper.py:490 with overlapping bed regions, or DCS_maker.py:258 with duplex keys that are not mutual)"; return CC_E_KEYERROR; }
    if (bits & EB_AMBIGUOUS) { ctx->err = "duplex keys are not mutual or span regions; reference outcome is order-dependent"; return CC_E_AMBIGUOUS; }
    if (bits & EB_N_HIGHQ) { ctx->err = "IndexError: N base with quality >= 30 in a family of size >= 2 (SSCS_maker.py:129)"; return CC_E_N_HIGHQ; }
    if (bits & EB_SHORT) { ctx->err = "IndexError: read shorter than the consensus length"; return CC_E_SHORT_READ; }
    if (bits & EB_BAD_BASE) { ctx->err = "ValueError: base outside ACGTN in a voted family (SSCS_maker.py:122)"; return CC_E_BAD_BASE; }
    if (bits & EB_NO_QUAL) { ctx->err = "TypeError: read without base qualities in a vote"; return CC_E_NO_QUAL; }
    if (bits & EB_NO_CIGAR) { ctx->err = "TypeError: infer_query_length() is None (no cigar)"; return CC_E_NO_CIGAR; }
    if (bits & EB_RG) { ctx->err = "RG tag of a non-string type"; return CC_E_UNSUPPORTED; }
    if (bits & EB_THR) { ctx->err = "cutoff table too short"; return CC_E_INVALID; }
    if (bits & EB_CHAIN) { ctx->err = "a chain of duplex partners longer than the engine follows"; return CC_E_UNSUPPORTED; }
    if (bits & EB_SCANWAIT) { ctx->err = "scan look-back wait bound exceeded"; return CC_E_INVALID; }
    if (bits & EB_TOO_LONG) { ctx->err = "record too long for the 16-bit length fields or payload > 64 GiB"; return CC_E_UNSUPPORTED; }
    ctx->err = "unknown device error";
    return CC_E_INVALID;
}

template <typename T>
int upload(cc_ctx* ctx, std::vector<void*>& allocs, T** dst, const T* src, int64_t count) {
    size_t bytes = (size_t)std::max<int64_t>(count, 1) * sizeof(T);
    HIPCHK(hipMalloc((void**)dst, bytes));
    allocs.push_back(*dst);
    if (count > 0) HIPCHK(hipMemcpyAsync(*dst, src, (size_t)count * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
    return 0;
}

#define GB(T, name, count) gbuf<T>(ctx, g, name, count, &brc); if (brc) return brc

int build_ht(cc_ctx* ctx, Group& g) {
    int brc = 0;
    uint64_t size = 1024;
    while (size < (uint64_t)(2 * g.F)) size <<= 1;
    g.ht_mask = size - 1;
    unsigned long long* key = GB(unsigned long long, "ht_key", (int64_t)size);
    int32_t* val = GB(int32_t, "ht_val", (int64_t)size);
    HIPCHK(hipMemsetAsync(key, 0xff, sizeof(unsigned long long) * size, ctx->stream));
    if (g.F > 0) {
        ProfScope ps(ctx, "k_ht_insert");
        hipLaunchKernelGGL(k_ht_insert, dim3(nblk(g.F)), dim3(256), 0, ctx->stream, g.F,
                           (const uint64_t*)g.buf["fam_hash"].p, key, val, g.ht_mask);
    }
    return 0;
}

// the barcode swap table (pageable host memory): copied only when it changed since the group's
// last upload, so a planned pass enqueues no pageable copy (that would wait for the stream)
int upload_swap(cc_ctx* ctx, Group& g, int32_t* d_swap, const int32_t* bc_swap, int32_t n_bc) {
    if (n_bc <= 0) return 0;
    if ((int32_t)g.swap_host.size() == n_bc && !memcmp(g.swap_host.data(), bc_swap, sizeof(int32_t) * n_bc)) return 0;
    g.swap_host.assign(bc_swap, bc_swap + n_bc);
    HIPCHK(hipMemcpyAsync(d_swap, bc_swap, sizeof(int32_t) * n_bc, hipMemcpyHostToDevice, ctx->stream));
    return 0;
}

PairView pair_view(Group& g) {
    return PairView{(const int32_t*)g.buf["pr_rec1"].p, (const int32_t*)g.buf["pr_rec2"].p,
                    (const int32_t*)g.buf["pr_region"].p, (const int32_t*)g.buf["region_run"].p, g.scoped,
                    (const int4*)g.buf["pr_tag"].p};
}

// the per-family tags of a grouping (k_fam_tags), built by the stages that join it (DCS, SC)
int ensure_fam_tags(cc_ctx* ctx, Group& g) {
    if (g.fam_tags_built) return 0;   // built by the pass (k_fam_build) or by an earlier join
    int brc = 0;
    TagKey* fam_tag = GB(TagKey, "fam_tag", g.F);
    int32_t* fam_rec = GB(int32_t, "fam_rec", g.F);
    g.fam_tags_built = true;
    if (g.F > 0) {
        ProfScope ps(ctx, "k_fam_tags");
        hipLaunchKernelGGL(k_fam_tags, dim3(nblk(g.F)), dim3(256), 0, ctx->stream, g.F,
                           (const int32_t*)g.buf["fam_first"].p, (const int32_t*)g.buf["fam_beg"].p,
                           (const int32_t*)g.buf["mem_rec"].p, pair_view(g), ctx->tables[g.table], fam_tag, fam_rec);
    }
    return 0;
}

GroupView view_of(Group& g) {
    GroupView v;
    v.F = g.F;
    v.seed = g.seed;
    v.ht_key = (const unsigned long long*)g.buf["ht_key"].p;
    v.ht_val = (const int32_t*)g.buf["ht_val"].p;
    v.ht_mask = g.ht_mask;
    v.fam_hash = (const uint64_t*)g.buf["fam_hash"].p;
    v.fam_first = (const int32_t*)g.buf["fam_first"].p;
    v.fam_beg = (const int32_t*)g.buf["fam_beg"].p;
    v.fam_region = (const int32_t*)g.buf["fam_region"].p;
    v.fam_o = (const int32_t*)g.buf["fam_o"].p;
    v.fam_tag = (const TagKey*)g.buf["fam_tag"].p;
    v.fam_rec = (const int32_t*)g.buf["fam_rec"].p;
    v.mem_rec = (const int32_t*)g.buf["mem_rec"].p;
    v.ent_f = (const int32_t*)g.buf["ent_f"].p;
    v.local = g.local_groups ? 1 : 0;
    v.fbkt = nullptr;
    v.tbase = nullptr;
    v.ntid = 0;
    v.geom = nullptr;
    return v;
}

// the family-bucket index of a local grouping over its table's position buckets (false: none)
int build_fam_buckets(cc_ctx* ctx, Group& g, GroupView* v, bool* ok) {
    *ok = false;
    const DevTable& T = ctx->tables[g.table];
    if (!g.local_groups || !g.coord_sorted) return 0;   // the table's buckets were built by g's pass
    int brc = 0;
    int32_t* fbkt = GB(int32_t, "fam_bkt", T.bkt_cap);
    {
        // the table's bucket geometry from each tid's extent (k_table_cols at upload)
        ProfScope ps(ctx, "k_bucket_geom");
        hipLaunchKernelGGL(k_bucket_geom, dim3(1), dim3(BG_T), 0, ctx->stream, T.n, T.ntid, (const int32_t*)T.ext,
                           T.tbase, T.geom);
    }
    hipLaunchKernelGGL(k_fam_bucket, dim3(nblk(g.F + 1)), dim3(256), 0, ctx->stream, g.F,
                       (const TagKey*)g.buf["fam_tag"].p, T.tbase, T.ntid,
                       T.geom, fbkt);
    v->fbkt = fbkt;
    v->tbase = T.tbase;
    v->ntid = T.ntid;
    v->geom = T.geom;
    *ok = true;
    return 0;
}

}  // namespace


extern "C" {

int cc_create(int device_id, cc_ctx** out) {
    if (!out) return CC_E_INVALID;
    std::unique_ptr<cc_ctx> c(new cc_ctx());
    cc_ctx* ctx = c.get();
    ctx->device = device_id;
    HIPCHK(hipSetDevice(device_id));
    HIPCHK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    HIPCHK(hipMalloc((void**)&ctx->d_err, 64));
    HIPCHK(hipMalloc((void**)&ctx->d_cnt, sizeof(unsigned long long) * CC_NUM_COUNTERS * CNT_STRIPES));
    HIPCHK(hipHostMalloc(&ctx->h_pinned, 1024 + sizeof(unsigned long long) * CC_NUM_COUNTERS * CNT_STRIPES));
    *out = c.release();
    return 0;
}

int cc_destroy(cc_ctx* ctx) {
    if (!ctx) return CC_E_INVALID;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& g : ctx->groups)
        for (auto& b : g.second->buf)
            if (b.second.p) (void)hipFree(b.second.p);
    for (auto& t : ctx->table_allocs)
        for (void* p : t.second) (void)hipFree(p);
    if (ctx->scratch)
        for (auto& b : ctx->scratch->buf)
            if (b.second.p) (void)hipFree(b.second.p);
    if (ctx->tmp.p) (void)hipFree(ctx->tmp.p);
    if (ctx->scan_st) (void)hipFree(ctx->scan_st);
    flush_prof(ctx);
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    (void)hipFree(ctx->d_err);
    (void)hipFree(ctx->d_cnt);
    (void)hipHostFree(ctx->h_pinned);
    if (ctx->h_defer) (void)hipHostFree(ctx->h_defer);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return 0;
}

const char* cc_last_error(cc_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void* cc_host_alloc(cc_ctx* ctx, uint64_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        if (ctx) ctx->err = "hipHostMalloc failed";
        return nullptr;
    }
    return p;
}
void cc_host_free(cc_ctx*, void* p) {
    if (p) (void)hipHostFree(p);
}

int cc_set_profiling(cc_ctx* ctx, int on) {
    if (!ctx) return CC_E_INVALID;
    flush_prof(ctx);
    ctx->profiling = on != 0;
    if (on) ctx->prof.clear();
    return 0;
}

int cc_profile_only(cc_ctx* ctx, const char* names) {
    if (!ctx) return CC_E_INVALID;
    ctx->prof_only.clear();
    if (!names) return 0;
    std::string all(names), cur;
    for (char c : all) {
        if (c == '\n') { if (!cur.empty()) ctx->prof_only.insert(cur); cur.clear(); }
        else cur.push_back(c);
    }
    if (!cur.empty()) ctx->prof_only.insert(cur);
    return 0;
}

int cc_kernel_times(cc_ctx* ctx, char* names, int names_cap, double* ms, int64_t* launches, int cap) {
    if (!ctx) return CC_E_INVALID;
    flush_prof(ctx);
    int i = 0;
    std::string all;
    for (auto& p : ctx->prof) {
        if (i < cap) {
            if (ms) ms[i] = p.second.ms;
            if (launches) launches[i] = p.second.n;
        }
        all += p.first;
        all.push_back('\n');
        ++i;
    }
    if (names && names_cap > 0) snprintf(names, names_cap, "%s", all.c_str());
    return i;
}

// Deferred end-of-pass checks (bench steps, batched stage calls): while on, a PLANNED pass does
// not wait for its readback; cc_commit waits once and judges every deferred pass.  A pass whose
// plan did not hold, that met an error or that needs the sort path makes cc_commit return
// CC_E_REPLAY: the caller runs the same calls again with deferral off (each then re-runs exactly
// where its plan failed and reports its own error).  Exact passes read back as usual.
int cc_defer(cc_ctx* ctx, int on) {
    if (!ctx) return CC_E_INVALID;
    if (!ctx->h_defer && on) {
        HIPCHK(hipHostMalloc((void**)&ctx->h_defer, (size_t)DEFER_SLOTS * DEFER_SLOT_BYTES));
        HIPCHK(hipHostGetDevicePointer((void**)&ctx->d_defer, ctx->h_defer, 0));
    }
    ctx->defer = on != 0;
    return 0;
}

int cc_commit(cc_ctx* ctx) {
    if (!ctx) return CC_E_INVALID;
    if (ctx->deferred.empty()) return 0;
    HIPCHK(stream_wait(ctx));
    if (const int rc = dbg_fault(ctx)) { ctx->deferred.clear(); return rc; }
    bool ok = true;
    for (const DeferredCheck& d : ctx->deferred) {
        if (!ctx->groups.count(d.gid) || ctx->groups[d.gid].get() != d.g) continue;   // freed since
        Group& g = *d.g;
        const uint8_t* h = ctx->h_defer + (size_t)d.slot * DEFER_SLOT_BYTES;
        if (*(const uint32_t*)h != 0) ok = false;   // an error, EB_PLAN or EB_NEEDSORT
        for (const auto& e : d.expect)
            if ((int64_t)((const uint32_t*)(h + 256))[e.first] != e.second) ok = false;
        if (d.counters) {
            for (int i = 0; i < CC_NUM_COUNTERS; ++i) {
                if (i == CC_CNT_COUNTER || i == CC_CNT_PAIRS || i == CC_CNT_READ_ENDS || i == CC_CNT_FAMILIES ||
                    i == CC_CNT_ENTRIES || i == CC_CNT_DROPPED)
                    continue;   // set by the pass from its (planned) totals
                g.counters[i] = (int64_t)((const unsigned long long*)(h + 1024))[i];   // summed (k_defer_pack)
            }
            g.counters[CC_CNT_COUNTER] = g.S - g.counters[CC_CNT_FOREIGN] - g.counters[CC_CNT_UNMAPPED];
        }
        // consensus_maker decides on the bad-read list from the counters it saw
        if (!d.counters && d.bad_listed != (g.counters[CC_CNT_BAD_LISTED] > 0)) ok = false;
    }
    ctx->deferred.clear();
    if (!ok) {
        ctx->err = "a deferred pass did not hold its plan or met an error: replay the calls with deferral off";
        return CC_E_REPLAY;
    }
    return 0;
}

// test hook: shifts one planned total of a group so that its next planned pass fails its check
// (exercises the exact re-run and the deferred replay)
int cc_debug_skew_plan(cc_ctx* ctx, int32_t group_id, const char* name, int64_t delta) {
    if (!ctx || !name || !ctx->groups.count(group_id)) return CC_E_INVALID;
    Group& g = *ctx->groups[group_id];
    if (!g.plan.count(name)) { ctx->err = std::string("no planned total named ") + name; return CC_E_INVALID; }
    g.plan[name] += delta;
    return 0;
}

int cc_synchronize(cc_ctx* ctx) {
    if (!ctx) return CC_E_INVALID;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    flush_prof(ctx);
    return dbg_fault(ctx);
}

int cc_debug_build(void) {
#ifdef CC_DEBUG_BOUNDS
    return 1;
#else
    return 0;
#endif
}

int64_t cc_launch_count(void) { return g_launches.load(std::memory_order_relaxed); }

int cc_table_upload(cc_ctx* ctx, const cc_records* r, int32_t max_len, int32_t* table_id) {
    if (!ctx || !r || !table_id) return CC_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    int32_t id = ctx->next_id++;
    std::vector<void*>& al = ctx->table_allocs[id];
    DevTable T;
    T.n = r->n;
    T.max_len = max_len;
    RC(upload(ctx, al, &T.tid, r->tid, r->n));
    RC(upload(ctx, al, &T.pos, r->pos, r->n));
    RC(upload(ctx, al, &T.mtid, r->mtid, r->n));
    RC(upload(ctx, al, &T.mpos, r->mpos, r->n));
    RC(upload(ctx, al, &T.tlen, r->tlen, r->n));
    RC(upload(ctx, al, &T.flag, r->flag, r->n));
    RC(upload(ctx, al, &T.mapq, r->mapq, r->n));
    RC(upload(ctx, al, &T.cig, r->cigar_id, r->n));
    RC(upload(ctx, al, &T.qlen, r->qlen, r->n));
    RC(upload(ctx, al, &T.lseq, r->lseq, r->n));
    RC(upload(ctx, al, &T.bc, r->bc_id, r->n));
    RC(upload(ctx, al, &T.rg, r->rg_id, r->n));
    RC(upload(ctx, al, &T.rflags, r->rflags, r->n));
    RC(upload(ctx, al, &T.qn_off, r->qn_off, r->n));
    RC(upload(ctx, al, &T.qn_len, r->qn_len, r->n));
    RC(upload(ctx, al, &T.qn_blob, r->qn_blob, (int64_t)r->qn_blob_bytes + 16));
    HIPCHK(hipMalloc((void**)&T.qn_ol, sizeof(uint64_t) * std::max<int64_t>(r->n, 1)));
    al.push_back(T.qn_ol);
    if (r->n > 0)
        hipLaunchKernelGGL(k_qn_pack, dim3(nblk(r->n)), dim3(256), 0, ctx->stream, r->n, (const uint64_t*)T.qn_off,
                           (const uint16_t*)T.qn_len, T.qn_ol);
    RC(upload(ctx, al, &T.pay_off, r->pay_off, r->n));
    RC(upload(ctx, al, &T.payload, r->payload, (int64_t)r->payload_bytes + 64));
    T.pay_bytes = r->payload_bytes;
    T.qn_bytes = r->qn_blob_bytes;
    if (!r->rdig) { ctx->err = "cc_records.rdig is required"; return CC_E_INVALID; }
    RC(upload(ctx, al, &T.rdig, r->rdig, r->n));
    HIPCHK(hipMalloc((void**)&T.core, sizeof(RecCore) * std::max<int64_t>(r->n, 1)));
    al.push_back(T.core);
    if (r->n > 0) hipLaunchKernelGGL(k_core_pack, dim3(nblk(r->n)), dim3(256), 0, ctx->stream, r->n, T);
    HIPCHK(hipMalloc((void**)&T.meta, sizeof(uint4) * std::max<int64_t>(r->n, 1)));
    al.push_back(T.meta);
    HIPCHK(hipMalloc((void**)&T.rkey, sizeof(uint64_t) * std::max<int64_t>(r->n, 1)));
    al.push_back(T.rkey);
    HIPCHK(hipMalloc((void**)&T.ebits, 16));
    al.push_back(T.ebits);
    HIPCHK(hipMemsetAsync(T.ebits, 0, 16, ctx->stream));
    // bucket geometry storage (filled per read_bam pass on a sorted table): sizes only, from the
    // largest tid; the bucket count is at most max(2N + ntid, 2 ntid) + 1 by k_bucket_geom's rule
    int32_t maxtid = -1;
    for (int64_t i = 0; i < r->n; ++i) maxtid = std::max(maxtid, r->tid[i]);
    T.ntid = maxtid + 1;
    T.bkt_cap = std::max<int64_t>(2 * r->n + T.ntid, 2 * (int64_t)T.ntid) + 2;
    HIPCHK(hipMalloc((void**)&T.ext, sizeof(int32_t) * std::max(T.ntid, 1)));
    al.push_back(T.ext);
    HIPCHK(hipMalloc((void**)&T.tbase, sizeof(int64_t) * (T.ntid + 1)));
    al.push_back(T.tbase);
    HIPCHK(hipMalloc((void**)&T.geom, 16));
    al.push_back(T.geom);
    HIPCHK(hipMemsetAsync(T.ext, 0, sizeof(int32_t) * std::max(T.ntid, 1), ctx->stream));
    if (r->n > 0) {
        ProfScope ps(ctx, "k_table_cols");
        hipLaunchKernelGGL(k_table_cols, dim3(nblk(r->n, BC_T)), dim3(BC_T), 0, ctx->stream, T);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));   // the uploads read caller memory
    ctx->tables[id] = T;
    *table_id = id;
    return 0;
}

}  // extern "C"

namespace {
// Per-pass table preparation (timed with the pass): the member records; on a coordinate-sorted table
// also the position keys, the read-end map and the bucket geometry.  No host synchronisation.
int prep_table(cc_ctx* ctx, const DevTable& T, bool coord, Fills& fill, int32_t* rec_e,
               int32_t* dlist = nullptr, uint32_t* ndeep = nullptr, int64_t dcap = 0) {
    RC(fill.launch());
    if (T.n <= 0) return 0;
    {
        ProfScope ps(ctx, "k_build_meta");
        hipLaunchKernelGGL(k_build_meta, dim3(nblk(T.n, BC_T)), dim3(BC_T), 0, ctx->stream, T, rec_e, ctx->d_err,
                           coord ? dlist : (int32_t*)nullptr, ndeep, dcap);
    }
    // (the bucket geometry from each tid's extent: built by the SC join that uses it, build_fam_buckets)
    return 0;
}
}  // namespace

extern "C" {

int cc_table_free(cc_ctx* ctx, int32_t id) {
    if (!ctx || !ctx->tables.count(id)) return CC_E_INVALID;
    (void)hipStreamSynchronize(ctx->stream);
    for (void* p : ctx->table_allocs[id]) (void)hipFree(p);
    ctx->table_allocs.erase(id);
    ctx->tables.erase(id);
    return 0;
}

}  // extern "C"

namespace {
// The SSCS vote (consensus_maker, SSCS_maker.py:81-168, with create_aligned_segment's fields) of the
// NE emitted families of group g: needv[o] flags the families that vote (size >= 2), vxs its
// exclusive scan (the vote slots), emit_fam / emit_span the family and its member range in
// g's member arrays (mem_meta, mem_rec, mem_valid, fam_beg/fam_end/fam_n).  Writes vote_fam,
// vote_meta, cons_seq and cons_qual of g; *NV_out = voted families.  Shared by cc_consensus_maker
// (families of a read_bam group) and cc_sscs_vote (families given by the caller).
int vote_families(cc_ctx* ctx, Group& g, const DevTable& T, int64_t NE, uint8_t* needv, uint32_t* vxs,
                  int32_t* emit_fam, int2* emit_span, double cutoff, int64_t* NV_out) {
    int brc = 0;
    int64_t NV = 0;
    RC(scan_total(ctx, g, needv, vxs, NE, &NV, "scan_vote"));
    g.NV = NV;
    g.Q = NE;
    int32_t* vote_fam = GB(int32_t, "vote_fam", NV);
    int4* vote_order = GB(int4, "vote_order", NV);
    int32_t* emit_vslot = GB(int32_t, "emit_vslot", NE);
    const int32_t qstride = (int32_t)((T.max_len + 15) & ~15);
    uint8_t* cons_seq = GB(uint8_t, "cons_seq", NV * (qstride / 2));
    uint8_t* cons_qual = GB(uint8_t, "cons_qual", NV * qstride);
    int32_t* vmeta = GB(int32_t, "vote_meta", 5 * NV);
    // families the SWAR vote cannot take (more than VOTE_BIGN members, or every family when reads
    // are longer than 64 SWAR chunks) land on a device-counted list for the split vote
    // (k_big_items / k_big_partial / k_big_final); their chunk count is a planned total
    const int32_t chunks = (T.max_len + SV_POS - 1) / SV_POS;
    const int all_slow = (chunks >= 1 && chunks <= 64) ? 0 : 1;
    int32_t* slow_list = GB(int32_t, "vote_slow_list", NV);
    uint32_t* d_items = (uint32_t*)(ctx->d_err) + 13;
    int brc2 = 0;
    uint32_t* d_nitems = plan_slot(ctx, g, "vote_items", &brc2);
    uint32_t* d_slow = plan_slot(ctx, g, "vote_slow", &brc2);   // families handed to the split vote
    if (brc2) return brc2;
    {
        // the error word and the hand-over counts (nothing before k_vote_plan reports errors)
        Fills fill(ctx);
        RC(fill.add(ctx->d_err, 64, 0u));
        RC(fill.add(d_nitems, 4, 0u));
        RC(fill.add(d_slow, 4, 0u));
        RC(fill.launch());
    }
    if (NE > 0) {
        ProfScope ps(ctx, "k_vote_plan");
        hipLaunchKernelGGL(k_vote_plan, dim3(nblk(NE)), dim3(256), 0, ctx->stream, NE, needv, vxs, emit_fam,
                           (const int2*)emit_span, (const uint4*)g.buf["mem_meta"].p, (const int32_t*)g.buf["mem_rec"].p, T, vote_fam,
                           vote_order, emit_vslot, vmeta, d_slow, slow_list, d_nitems, all_slow, ctx->d_err);
    }
    if (NV > 0) {
        int64_t NI = 0, NSL = 0;
        RC(planned_total(ctx, g, "vote_items", d_nitems, &NI));
        RC(planned_total(ctx, g, "vote_slow", d_slow, &NSL));
        if (!all_slow) {
            const bool fresh = !g.buf.count("cutoff_thr") || !g.buf["cutoff_thr"].p;
            int32_t* thr = GB(int32_t, "cutoff_thr", VOTE_BIGN + 1);
            if (fresh || g.thr_cutoff != cutoff) {   // the table depends on the cutoff alone
                hipLaunchKernelGGL(k_cutoff_table, dim3(1), dim3(128), 0, ctx->stream, cutoff, thr);
                g.thr_cutoff = cutoff;
            }
            const int32_t fpw = 64 / chunks;
            const int64_t waves = (NV + fpw - 1) / fpw;
            const int32_t uni_ok = (1.0 >= cutoff) ? 1 : 0;   // count == pass: 1.0 >= cutoff in double
            ProfScope ps(ctx, "k_sscs_vote_swar");
            hipLaunchKernelGGL(k_sscs_vote_swar, dim3(nblk(waves, 4)), dim3(256), 0, ctx->stream, NV, fpw, chunks,
                               vote_order, (const uint4*)g.buf["mem_meta"].p, T, thr, uni_ok, qstride, cons_seq,
                               cons_qual, ctx->d_err);
        }
        const int64_t icap = NI > 0 ? NI : 1;
        int32_t* big_item = GB(int32_t, "vote_big_item", NV);
        int4* items = GB(int4, "vote_items", icap);
        uint8_t* partial = GB(uint8_t, "vote_partial", icap * BIG_PL * (int64_t)qstride);
        if (NSL > 0) {
            ProfScope ps(ctx, "k_big_items");
            hipLaunchKernelGGL(k_big_items, dim3(64), dim3(256), 0, ctx->stream, d_slow, slow_list, vote_fam,
                               (const int32_t*)g.buf["fam_beg"].p, (const int32_t*)g.buf["fam_end"].p, NI, d_items,
                               big_item, items, ctx->d_err);
        }
        if (NI > 0) {
            const int32_t bch = std::min(64, std::max(1, (T.max_len + SV_POS - 1) / SV_POS));   // lanes per item
            const int32_t bfpw = 64 / bch;
            ProfScope ps(ctx, "k_big_swar");
            hipLaunchKernelGGL(k_big_swar, dim3(nblk((NI + bfpw - 1) / bfpw, 4)), dim3(256), 0, ctx->stream, d_items, NI,
                               bfpw, bch, items, (const uint4*)g.buf["mem_meta"].p, T, qstride, partial, ctx->d_err);
        }
        ProfScope ps(ctx, "k_big_final");
        if (NSL > 0)
        hipLaunchKernelGGL(k_big_final, dim3(8192), dim3(64), 0, ctx->stream, d_slow, slow_list, big_item, NI,
                           vote_fam, (const int32_t*)g.buf["fam_beg"].p, (const int32_t*)g.buf["fam_end"].p,
                           (const int32_t*)g.buf["fam_n"].p, (const int32_t*)g.buf["mem_rec"].p,
                           (const uint32_t*)g.buf["mem_valid"].p, (const uint4*)g.buf["mem_meta"].p, T, cutoff,
                           qstride, partial, qstride, cons_seq, cons_qual, vmeta, ctx->d_err);
    }
    *NV_out = NV;
    return 0;
}
}  // namespace

// ------------------------------------------------------------------ read_bam pipeline
namespace {

int read_bam_pass(cc_ctx* ctx, int32_t gid) {
    Group& g = *ctx->groups[gid];
    const DevTable& T = ctx->tables[g.table];
    const int64_t S = g.S;
    int brc = 0;
    int32_t* d_srec = (int32_t*)g.buf["stream_rec"].p;
    int32_t* d_sreg = (int32_t*)g.buf["stream_region"].p;
    int32_t* d_run = (int32_t*)g.buf["region_run"].p;
    uint32_t* d_nresid = plan_slot(ctx, g, "n_resid", &brc);       // count-only totals (wave atomics)
    uint32_t* d_nbig = plan_slot(ctx, g, "n_big", &brc);
    uint32_t* d_ndrop = plan_slot(ctx, g, "n_drop", &brc);
    if (brc) return brc;
    const bool coord = g.coord_sorted && S > 0;             // sorted table: position-group grouping
    const bool coord_pair = coord && !g.force_sort;         // and the mate search by coordinates
    // the votes' member records: written as the ends are ranked by the pass whose stage votes
    // families (the SSCS stage's, the one that lists bad reads); built on demand otherwise
    const bool members = g.badread != 0;
    g.members_built = false;
    // the long pairs' keys (k_pair_coord_tile, k_pair_resid): at least twice the long pairs of the last
    // exact pass (deep groups' pairs are long), an exact pass room for every pair; more long pairs
    // than fit send the pass to the sort path
    uint32_t* n_long = plan_slot(ctx, g, "n_long", &brc);
    if (brc) return brc;
    uint64_t lsize = 1 << 10;
    {
        const uint64_t want = g.fast && g.plan.count("n_long") ? (uint64_t)(2 * g.plan["n_long"]) + (uint64_t)S / 16
                                                               : (uint64_t)S;
        while (lsize < want) lsize <<= 1;
    }
    unsigned long long* ltab = nullptr;
    if (coord_pair) ltab = GB(unsigned long long, "pc_ltab", (int64_t)lsize);
    // the pass's zeroed words, one launch with the table preparation's
    Fills fill(ctx);
    RC(fill.add(ctx->d_err, 4, 0u));
    RC(fill.add(ctx->d_cnt, sizeof(unsigned long long) * CC_NUM_COUNTERS * CNT_STRIPES, 0u));
    RC(fill.add(g.buf["plan_totals"].p, 4 * PLAN_SLOTS, 0u));
    // every striped count starts the pass at zero (k_stripe_total zeroes what it folds; a planned
    // pass's unfolded stripes are summed at its end, and a pass that ended early leaves them set)
    if (g.buf.count("plan_stripes") && g.buf["plan_stripes"].p)
        RC(fill.add(g.buf["plan_stripes"].p, sizeof(uint32_t) * PLAN_SLOTS * PSTRIPES * PSTRIDE, 0u));
    g.stripes_pending = false;
    if (ltab) RC(fill.add(ltab, sizeof(unsigned long long) * lsize, ~0u));
    // a planned pass knows its family count: the per-family drop counts are zeroed here too
    bool drop_zeroed = false;
    if (g.fast && g.plan.count("scan_fam") && g.plan["scan_fam"] > 0) {
        int32_t* fd = GB(int32_t, "fam_drop", g.plan["scan_fam"]);
        RC(fill.add(fd, sizeof(int32_t) * g.plan["scan_fam"], 0u));
        drop_zeroed = true;
    }
    // a bed stream's keys and slots scattered to its records (k_scatter_stream) for the mate search;
    // records outside the stream keep the all-ones fill (key ~0, slot -1)
    uint64_t* rq = nullptr;    // identity streams read the stream keys instead
    int32_t* spos = nullptr;   // and a record index as the stream slot
    if (coord_pair && !g.ident) {
        rq = GB(uint64_t, "pc_rq", T.n);
        spos = GB(int32_t, "pc_spos", T.n);
        RC(fill.add(rq, sizeof(uint64_t) * T.n, ~0u));
        RC(fill.add(spos, sizeof(int32_t) * T.n, ~0u));
    }
    // ---- 0. the table's per-record cores (and position keys when sorted), part of every pass
    int32_t* pre = nullptr;
    if (g.coord_sorted && T.n > 0) { pre = GB(int32_t, "rec_e", T.n); }
    // the deep position groups' first records (k_build_meta), for the per-group sorts
    uint32_t* d_ndg = plan_slot(ctx, g, "n_deepg", &brc);
    if (brc) return brc;
    const int64_t dcap = T.n / DEEP_MIN + 2;
    int32_t* dlist = nullptr;
    if (g.coord_sorted && T.n > 0) { dlist = GB(int32_t, "deep_list", dcap); }
    // ---- 1. filters + qname keys (consensus_helper.py:389-426)
    uint64_t* skey = GB(uint64_t, "skey", S);
    uint32_t* sval = GB(uint32_t, "sval", S);
    uint64_t* skey2 = GB(uint64_t, "skey2", S);
    uint32_t* sval2 = GB(uint32_t, "sval2", S);
    uint8_t* badflag = GB(uint8_t, "badflag", (S + 15) & ~15LL);   // byte flags (16-B padded for the scan)
    int32_t* mate_of = GB(int32_t, "mate_of", S);
    uint8_t* pflag = GB(uint8_t, "pflag", (S + 15) & ~15LL);
    const int64_t N = T.n;
    int32_t* partner = nullptr;
    int32_t* claims = nullptr;
    if (coord_pair) {
        partner = GB(int32_t, "pc_partner", S);
        claims = GB(int32_t, "pc_claims", S);
    }
    const ClassifyOut co{skey, coord_pair ? nullptr : sval, g.badread ? badflag : nullptr, mate_of,
                         g.ident ? nullptr : partner, claims, pflag};
    // an identity stream on a sorted table: the table preparation and the filters in one pass over
    // the records (k_build_meta_cls); otherwise the preparation, then the stream's filters
    const bool fused = g.ident && coord_pair && S == T.n && T.n > 0;
    if (fused) {
        RC(fill.launch());
        {
            ProfScope ps(ctx, "k_build_meta_cls");
            hipLaunchKernelGGL(k_build_meta_cls, dim3(nblk(T.n, BC_T)), dim3(BC_T), 0, ctx->stream, T, pre,
                               ctx->d_err, dlist, d_ndg, dcap, (const int32_t*)d_sreg, (const int32_t*)d_run,
                               g.delim_filter, g.badread, g.scoped, g.seed, co, ctx->d_cnt);
        }
    } else {
        RC(prep_table(ctx, T, g.coord_sorted != 0, fill, pre, dlist, d_ndg, dcap));
        if (S > 0) {
            ProfScope ps(ctx, "k_classify");
            hipLaunchKernelGGL(k_classify, dim3(nblk(S)), dim3(256), 0, ctx->stream, S, g.ident, d_srec, d_sreg, d_run, T,
                               g.delim_filter, g.badread, g.scoped, g.seed, co, ctx->d_cnt);
        }
    }
    int64_t NDG = 0;
    if (dlist) RC(planned_total(ctx, g, "n_deepg", d_ndg, &NDG));
    g.n_deepg = NDG;
    uint32_t* deep_gid = nullptr;   // per record its deep group (k_deep_qsort), for the deep tag sort
    // ---- 2. pair_dict: mates by qname
    uint32_t* d_nmulti = plan_slot(ctx, g, "n_multi", &brc);   // qnames seen more than twice (k_pair_mark)
    if (brc) return brc;
    bool sorted_pairing = false;   // k_pair_mark ran (the only source of n_multi)
    if (coord) {
        uint64_t* rkey = T.rkey;   // (the table's position keys, k_table_cols)
        int32_t* rec_e = GB(int32_t, "rec_e", N);
        ProfScope ps(ctx, "k_pair_coord");
        if (coord_pair) {
            uint8_t* resid = GB(uint8_t, "pc_resid", (S + 15) & ~15LL);   // byte flags (16-B padded for the scan)
            if (!g.ident)
                hipLaunchKernelGGL(k_scatter_stream, dim3(nblk(S)), dim3(256), 0, ctx->stream, S, g.ident, d_srec, skey, spos, rq);
            const uint64_t* qk = g.ident ? (const uint64_t*)skey : (const uint64_t*)rq;
            // deep position groups: each group's records sorted by qname key (the search bisects there)
            uint64_t* gq = nullptr;
            int32_t* gend = nullptr;
            uint32_t* boff = nullptr;
            unsigned long long* dgk = nullptr;   // 16-B entries (dg_insert)
            uint64_t dgsize = 64;
            if (NDG > 0) {
                while (dgsize < (uint64_t)(2 * NDG)) dgsize <<= 1;
                gq = GB(uint64_t, "deep_gq", N);
                gend = GB(int32_t, "deep_gend", N);
                boff = GB(uint32_t, "deep_boff", N + 1);
                deep_gid = GB(uint32_t, "deep_gid", N);
                dgk = GB(unsigned long long, "deep_dgk", 2 * (int64_t)dgsize);
                RC(fill.add(dgk, sizeof(unsigned long long) * 2 * dgsize, 0xFFFFFFFEu));
                RC(fill.launch());
                ProfScope pq(ctx, "k_deep_qsort");
                hipLaunchKernelGGL(k_deep_qsort, dim3((unsigned)std::min<int64_t>(NDG, 1024)), dim3(DQ_T), 0, ctx->stream,
                                   (const uint32_t*)d_ndg, (const int32_t*)dlist, N, (const uint64_t*)rkey, qk, gq, gend,
                                   boff, dgk, dgsize - 1, deep_gid);
            }
            uint32_t* lst = plan_stripes(ctx, g, n_long, &brc);
            if (brc) return brc;
            // the search runs over the table's records (coordinate order) with their qname keys staged
            // in LDS per tile: the stream keys themselves on an identity stream, else scattered to the
            // records by k_scatter_stream (rq, and each record's stream slot spos)
            const char* pct = getenv("CC_PC_TILE");   // 512 / 1024: force a tile size (measurements)
            const bool small = pct ? atoi(pct) == 512 : N < PC_SMALL_N;
            if (small)
                hipLaunchKernelGGL(k_pair_coord_tile<512>, dim3(nblk(N, 512)), dim3(256), 0, ctx->stream, N, qk,
                                   g.ident ? (const int32_t*)nullptr : (const int32_t*)spos, rkey, T, partner, claims,
                                   mate_of, pflag, ltab, lsize - 1, lst, ctx->d_err, (const uint64_t*)gq,
                                   (const int32_t*)gend, (const uint32_t*)boff, (const unsigned long long*)dgk,
                                   dgsize - 1);
            else
                hipLaunchKernelGGL(k_pair_coord_tile<1024>, dim3(nblk(N, 1024)), dim3(256), 0, ctx->stream, N, qk,
                                   g.ident ? (const int32_t*)nullptr : (const int32_t*)spos, rkey, T, partner, claims,
                                   mate_of, pflag, ltab, lsize - 1, lst, ctx->d_err, (const uint64_t*)gq,
                                   (const int32_t*)gend, (const uint32_t*)boff, (const unsigned long long*)dgk,
                                   dgsize - 1);
            hipLaunchKernelGGL(k_stripe_total, dim3(1), dim3(64), 0, ctx->stream, lst, n_long);
            uint32_t* st = plan_stripes(ctx, g, d_nresid, &brc);
            if (brc) return brc;
            hipLaunchKernelGGL(k_pair_resid, dim3((unsigned)((S + PD_TILE - 1) / PD_TILE)), dim3(256), 0, ctx->stream, S,
                               skey, partner, claims, resid, st, ltab, lsize - 1, n_long, ctx->d_err);
            // a planned pass leaves the count striped: the end-of-pass check folds it (k_defer_pack)
            if (g.fast && g.plan.count("n_resid")) g.stripes_pending = true;
            else hipLaunchKernelGGL(k_stripe_total, dim3(1), dim3(64), 0, ctx->stream, st, d_nresid);
        }
    }
    if (coord_pair) {
        int64_t NL = 0;   // the long pairs: the next planned pass sizes its table from them
        RC(planned_total(ctx, g, "n_long", n_long, &NL));
        const uint8_t* resid = (const uint8_t*)g.buf["pc_resid"].p;
        int64_t NR = 0;
        RC(planned_total(ctx, g, "n_resid", d_nresid, &NR));
        if (NR > 0) {
            // residual reads (mate not found by coordinates): a qname paired by coordinates must not also
            // be residual (3+ occurrences), then the exact sort path pairs the residual reads.  Their
            // keys are compacted in the scan of the byte flags (EmitResid), which also fills the exact
            // table and its Bloom filter that the other entries probe (k_resid_probe); with many residual
            // reads (more than a quarter of the stream) the sorted keys are searched instead
            const bool many = NR > S / 4;
            uint64_t hsize = 1024, bsize = 1024;
            while (!many && hsize < (uint64_t)(2 * NR)) hsize <<= 1;
            while (!many && bsize < (uint64_t)(NR / 4 + 1)) bsize <<= 1;   // 16 filter bits per key
            unsigned long long* rht = nullptr;
            unsigned long long* bloom = nullptr;
            uint32_t *hcnt = nullptr, *hmin = nullptr, *hmax = nullptr;
            uint32_t* d_rmulti = plan_slot(ctx, g, "resid_multi", &brc);
            if (brc) return brc;
            if (!many) {
                rht = GB(unsigned long long, "pc_rht", (int64_t)hsize);
                bloom = GB(unsigned long long, "pc_bloom", (int64_t)bsize);
                hcnt = GB(uint32_t, "pc_hcnt", (int64_t)hsize);
                hmin = GB(uint32_t, "pc_hmin", (int64_t)hsize);
                hmax = GB(uint32_t, "pc_hmax", (int64_t)hsize);
                RC(fill.add(rht, sizeof(unsigned long long) * hsize, ~0u));
                RC(fill.add(bloom, sizeof(unsigned long long) * bsize, 0u));
                RC(fill.add(hcnt, sizeof(uint32_t) * hsize, 0u));
                RC(fill.add(hmin, sizeof(uint32_t) * hsize, ~0u));
                RC(fill.add(hmax, sizeof(uint32_t) * hsize, 0u));
                RC(fill.launch());
            }
            uint64_t* rk = GB(uint64_t, "pc_rk", NR);
            uint32_t* rv = GB(uint32_t, "pc_rv", NR);
            int64_t NR2 = 0;
            RC(scan_emit(ctx, g, resid, S, &NR2, "scan_resid",
                         EmitResid{skey, rk, rv, NR, rht, hsize - 1, bloom, bsize - 1, ctx->d_err, hcnt, hmin, hmax,
                                   d_rmulti}));
            if (!many) {
                ProfScope ps(ctx, "k_pair_resid");
                hipLaunchKernelGGL(k_resid_probe, dim3(nblk(S)), dim3(256), 0, ctx->stream, S, skey, resid,
                                   (const unsigned long long*)rht, hsize - 1, (const unsigned long long*)bloom, bsize - 1,
                                   ctx->d_err);
            }
            int64_t nmulti_r = 1;
            if (!many) RC(planned_total(ctx, g, "resid_multi", d_rmulti, &nmulti_r));
            if (!many && nmulti_r == 0 && !getenv("CC_RESID_SORT")) {
                // every residual key seen once or twice: paired through the table, no sort
                ProfScope ps(ctx, "k_pair_mark");
                hipLaunchKernelGGL(k_resid_pair, dim3(nblk(NR)), dim3(256), 0, ctx->stream, NR, (const uint64_t*)rk,
                                   (const uint32_t*)rv, (const unsigned long long*)rht, hsize - 1, (const uint32_t*)hcnt,
                                   (const uint32_t*)hmin, (const uint32_t*)hmax, g.ident, d_srec, T, mate_of, pflag,
                                   ctx->d_err, ctx->d_cnt);
            } else {
            RC(sort_pairs(ctx, rk, skey2, rv, sval2, NR, "sort_qname_resid"));
            if (many) {
                ProfScope ps(ctx, "k_pair_resid");
                hipLaunchKernelGGL(k_resid_probe_sorted, dim3(nblk(S)), dim3(256), 0, ctx->stream, S, skey, resid,
                                   (const uint64_t*)skey2, NR, ctx->d_err);
            }
            ProfScope ps(ctx, "k_pair_mark");
            uint32_t* mst = plan_stripes(ctx, g, d_nmulti, &brc);
            if (brc) return brc;
            hipLaunchKernelGGL(k_pair_mark, dim3(nblk(NR)), dim3(256), 0, ctx->stream, NR, skey2, sval2, g.ident, d_srec, T,
                               mate_of, pflag, ctx->d_err, ctx->d_cnt, mst);
            sorted_pairing = true;
            hipLaunchKernelGGL(k_stripe_total, dim3(1), dim3(64), 0, ctx->stream, mst, d_nmulti);
            }
        }
    } else {
        RC(sort_pairs(ctx, skey, skey2, sval, sval2, S, "sort_qname"));
        if (S > 0) {
            ProfScope ps(ctx, "k_pair_mark");
            uint32_t* mst = plan_stripes(ctx, g, d_nmulti, &brc);
            if (brc) return brc;
            hipLaunchKernelGGL(k_pair_mark, dim3(nblk(S)), dim3(256), 0, ctx->stream, S, skey2, sval2, g.ident, d_srec, T,
                               mate_of, pflag, ctx->d_err, ctx->d_cnt, mst);
            sorted_pairing = true;
            hipLaunchKernelGGL(k_stripe_total, dim3(1), dim3(64), 0, ctx->stream, mst, d_nmulti);
        }
    }
    // ---- 3. completed pairs (records, region, read ends) and their unique_tag / sscs_qname hashes
    int64_t P = 0;
    int32_t* pr_rec1 = GB(int32_t, "pr_rec1", S);   // capacity; sized P below
    int32_t* pr_rec2 = GB(int32_t, "pr_rec2", S);
    int32_t* pr_region = GB(int32_t, "pr_region", S);
    RC(scan_emit(ctx, g, pflag, S, &P, "scan_pairs",
                 EmitPairs{mate_of, g.ident, d_srec, d_sreg, pr_rec1, pr_rec2, pr_region,
                           g.coord_sorted ? (int32_t*)g.buf["rec_e"].p : nullptr}));
    g.P = P;
    pr_rec1 = GB(int32_t, "pr_rec1", P);
    pr_rec2 = GB(int32_t, "pr_rec2", P);
    pr_region = GB(int32_t, "pr_region", P);
    int4* pr_tag = GB(int4, "pr_tag", P);
    const PairView PV{pr_rec1, pr_rec2, pr_region, d_run, g.scoped, pr_tag};
    const int64_t R = 2 * P;
    g.R = R;
    uint64_t* chash = GB(uint64_t, "chash", P);
    uint64_t* thash = nullptr, *rhash = nullptr;   // tag hashes by read end (sort path) or by record
    if (g.coord_sorted) { rhash = GB(uint64_t, "rec_thash", N); }
    else { thash = GB(uint64_t, "thash", R); }
    uint32_t* tval = g.coord_sorted ? nullptr : GB(uint32_t, "tval", R);   // the tag sort's values
    uint64_t* rs_key = GB(uint64_t, "rs_key", R);
    uint32_t* rs_val = GB(uint32_t, "rs_val", R);
    uint8_t* cflag = GB(uint8_t, "cflag", (R + 15) & ~15LL);
    uint32_t* bigE = nullptr;
    if (g.coord_sorted && R > 0) {
        bigE = GB(uint32_t, "grp_bigE", R);
        RC(fill.add(bigE, sizeof(uint32_t) * R, 0u));
    }
    if (R > 0) RC(fill.add(cflag, ((size_t)R + 15) & ~(size_t)15, 0u));
    RC(fill.launch());
    if (P > 0) {
        ProfScope ps(ctx, "k_pair_keys");
        hipLaunchKernelGGL(k_pair_keys, dim3(nblk(P)), dim3(256), 0, ctx->stream, P, PV, T, g.seed, chash, thash,
                           tval, pr_tag, rhash);
    }
    // ---- 4. read_dict / tag_dict: group read ends by exact tag
    g.local_groups = false;
    int32_t* mem_rec = GB(int32_t, "mem_rec", R);
    int64_t n_known = 0;   // mem_rec[0, n_known) written by k_group_rank
    int64_t n_deep = 0;    // read ends in deep position groups
    bool deep_same_group = false;   // their sort keys are group-major (equal keys: one position group)
    bool deep_ranked = false;       // k_deep_fam ranked them (no sort, no k_fam_mark)
    if (g.coord_sorted && R > 0) {
        int32_t* rec_e = (int32_t*)g.buf["rec_e"].p;      // initialised by k_build_meta
        const uint64_t* rkey = (const uint64_t*)T.rkey;   // the table's position keys (k_table_cols)
        const int64_t NT = (N + GT - 1) / GT;
        uint32_t* tsmall = GB(uint32_t, "grp_tile_small", NT);
        {
            ProfScope ps(ctx, "k_group");
            uint32_t* st = plan_stripes(ctx, g, d_nbig, &brc);
            if (brc) return brc;
            hipLaunchKernelGGL(k_group_flags, dim3(nblk(N, GT)), dim3(GT), 0, ctx->stream, N, rkey, rec_e, tsmall, bigE,
                               st);
            if (g.fast && g.plan.count("n_big")) g.stripes_pending = true;
            else hipLaunchKernelGGL(k_stripe_total, dim3(1), dim3(64), 0, ctx->stream, st, d_nbig);
        }
        int64_t NS = 0, NB = 0;
        uint32_t* tpre = GB(uint32_t, "grp_tile_pre", NT);
        RC(scan_total(ctx, g, tsmall, tpre, NT, &NS, "scan_small"));
        if (NS > 0) {
            ProfScope ps(ctx, "k_group_rank");
            uint8_t* segf0 = GB(uint8_t, "segf", (R + 15) & ~15LL);
            uint32_t* valid0 = GB(uint32_t, "mem_valid", R);
            uint4* meta0 = nullptr;
            if (members) { meta0 = GB(uint4, "mem_meta", R); }
            hipLaunchKernelGGL(k_group_rank, dim3(nblk(N, GT)), dim3(GT), 0, ctx->stream, N, rkey, rec_e,
                               (const uint64_t*)rhash, (const uint32_t*)tpre, rs_key, rs_val, mem_rec, PV, T, segf0,
                               valid0, meta0, ctx->d_err);
        }
        n_known = NS;
        RC(planned_total(ctx, g, "n_big", d_nbig, &NB));
        n_deep = NB;
        if (NS + NB != R) {
            // inconsistent coordinate pairs (a record paired twice) lose read ends here; the qname
            // check that sends such a pass to the sort path has flagged it by now
            uint32_t eb = 0;
            RC(read_err(ctx, &eb));
            if (eb & EB_NEEDSORT) return CC_E_NEEDSORT;
            ctx->err = "position-group partition lost read ends";
            return CC_E_INVALID;
        }
        g.local_groups = NB == 0;
        if (NB > 0 && deep_gid && NDG > 0 && !g.no_deep_fam && !getenv("CC_DEEP_SORT")) {
            // the deep groups ranked in place (k_deep_fam, k_deep_emit, k_deep_sortfam): no global sort
            const int32_t* gend = (const int32_t*)g.buf["deep_gend"].p;
            uint32_t* gcnt = GB(uint32_t, "deep_gcnt", NDG);
            uint32_t* goff = GB(uint32_t, "deep_goff", NDG);
            uint32_t* se = GB(uint32_t, "deep_se", N);
            int4* items = GB(int4, "deep_items", NB);
            int4* bigit = GB(int4, "deep_big", NB / 65 + 1);
            uint32_t* d_ovf = plan_slot(ctx, g, "deep_ovf", &brc);
            if (brc) return brc;
            uint32_t* d_items = plan_slot(ctx, g, "deep_items", &brc);
            if (brc) return brc;
            uint32_t* d_big = plan_slot(ctx, g, "deep_big", &brc);
            if (brc) return brc;
            uint8_t* segf1 = GB(uint8_t, "segf", (R + 15) & ~15LL);
            uint32_t* valid1 = GB(uint32_t, "mem_valid", R);
            uint4* meta1 = nullptr;
            if (members) { meta1 = GB(uint4, "mem_meta", R); }
            const DeepOut dout{R, rs_val, mem_rec, segf1, valid1, meta1};
            {
                ProfScope ps(ctx, "k_deep_count");
                hipLaunchKernelGGL(k_deep_count, dim3((unsigned)std::min<int64_t>(NDG, 4096)), dim3(256), 0, ctx->stream,
                                   (const uint32_t*)d_ndg, (const int32_t*)dlist, gend, (const int32_t*)rec_e, gcnt);
            }
            int64_t nd = 0;
            RC(scan_total(ctx, g, gcnt, goff, NDG, &nd, "scan_deep"));
            if (nd != NB) {
                ctx->err = "deep position groups: end count differs from the group partition";
                return CC_E_INVALID;
            }
            {
                ProfScope ps(ctx, "k_deep_fam");
                hipLaunchKernelGGL(k_deep_fam, dim3((unsigned)std::min<int64_t>(NDG, 4096)), dim3(DF_T), 0, ctx->stream,
                                   (const uint32_t*)d_ndg, (const int32_t*)dlist, gend, (const int32_t*)rec_e,
                                   (const uint64_t*)rhash, (const uint32_t*)goff, NS, PV, T, se, items, d_items, bigit,
                                   d_big, d_ovf, ctx->d_err);
            }
#ifdef DF_PROF
            {
                unsigned long long hp[8];
                HIPCHK(hipStreamSynchronize(ctx->stream));
                HIPCHK(hipMemcpyFromSymbol(hp, HIP_SYMBOL(g_df_prof), sizeof(hp)));
                fprintf(stderr, "[deep_fam] NDG %lld  block-us: table %.0f numbering %.0f place %.0f\n", (long long)NDG,
                        hp[0] / 100.0, hp[1] / 100.0, hp[2] / 100.0);
                memset(hp, 0, sizeof(hp));
                HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_df_prof), hp, sizeof(hp)));
            }
#endif
            int64_t novf = 0;
            RC(planned_total(ctx, g, "deep_ovf", d_ovf, &novf));
            if (novf == 0) {
                {
                    ProfScope ps(ctx, "k_deep_emit");
                    hipLaunchKernelGGL(k_deep_emit, dim3((unsigned)std::min<int64_t>(NB / 256 + 1, 8192)), dim3(256), 0,
                                       ctx->stream, (const int4*)items, (const uint32_t*)d_items, (const uint32_t*)se, PV,
                                       T, dout, ctx->d_err);
                }
                int64_t nbig = 0;
                RC(planned_total(ctx, g, "deep_big", d_big, &nbig));
                if (nbig > 0) {
                    ProfScope ps(ctx, "k_deep_sortfam");
                    hipLaunchKernelGGL(k_deep_sortfam, dim3((unsigned)std::min<int64_t>(nbig, 2048)), dim3(DF_ST), 0,
                                       ctx->stream, (const int4*)bigit, (const uint32_t*)d_big, (const uint32_t*)se, PV, T,
                                       dout, ctx->d_err);
                }
                deep_ranked = true;
            }
        }
        if (NB > 0 && !deep_ranked) {
            uint32_t* bx = GB(uint32_t, "grp_bx", R);
            RC(scan_total(ctx, g, bigE, bx, R, &NB, "scan_bigE"));
            uint64_t* bkey = GB(uint64_t, "grp_bkey", NB);
            uint32_t* bval = GB(uint32_t, "grp_bval", NB);
            // group-major keys when this pass's coordinate search numbered the deep groups
            // (k_deep_qsort), else the full tag hash.  (The same keys with the hash bits in 16..63 and
            // a sort over bits 16..63 split c4 families on the GPU: rocPRIM's begin_bit is not used.)
            int gbits = 1;
            while ((1LL << gbits) < NDG) ++gbits;
            const char* kbe = getenv("CC_DEEP_KEYBITS");
            const int kb = kbe ? atoi(kbe) : 48;
            const bool by_group = deep_gid != nullptr && kb > 0 && gbits <= 24;
            deep_same_group = by_group;
            hipLaunchKernelGGL(k_big_keys, dim3(nblk(R)), dim3(256), 0, ctx->stream, R, bigE, bx,
                               (const uint64_t*)rhash, PV, (const uint32_t*)(by_group ? deep_gid : nullptr), gbits,
                               by_group ? kb : 64, bkey, bval);
            RC(sort_pairs(ctx, bkey, rs_key + NS, bval, rs_val + NS, NB, "sort_tags_big", 0u, by_group ? (unsigned)kb : 64u));
        }
    } else {
        RC(sort_pairs(ctx, thash, rs_key, tval, rs_val, R, "sort_tags"));
    }
    uint8_t* segf = GB(uint8_t, "segf", (R + 15) & ~15LL);
    uint32_t* validf = GB(uint32_t, "mem_valid", R);
    uint4* mem_meta = nullptr;
    if (members) { mem_meta = GB(uint4, "mem_meta", R); }
    if (R > 0) {
        ProfScope ps(ctx, "k_fam_mark");
        // the small groups' slots [0, n_known) were marked by k_group_rank
        if (R > n_known && !deep_ranked)
            hipLaunchKernelGGL(k_fam_mark, dim3(nblk(R - n_known)), dim3(256), 0, ctx->stream, R, n_known, n_known, rs_key,
                               rs_val, PV, T, segf, validf, mem_rec, mem_meta, ctx->d_err, deep_same_group ? 1 : 0);
        // qnames seen more than twice exist only where the exact pairing (k_pair_mark) ran this pass
        if (sorted_pairing)
        hipLaunchKernelGGL(k_fam_dedup, dim3(std::min<unsigned>(nblk(R), 1024u)), dim3(256), 0, ctx->stream, R,
                           (const uint32_t*)d_nmulti, (const uint8_t*)segf, validf, (const int32_t*)mem_rec,
                           (const uint32_t*)rs_val, (const int32_t*)pr_rec1, (const uint64_t*)T.rdig, mem_meta);
    }
    // family starts compacted in the scan's store phase (EmitFamStarts): fam_beg and fam_drop take
    // their capacity first (F is the scan's total)
    int64_t F = 0, V = 0;
    const int64_t Fcap = g.fast && g.plan.count("scan_fam") ? g.plan["scan_fam"] : R;
    int32_t* fam_beg = GB(int32_t, "fam_beg", Fcap);
    int32_t* fam_drop = GB(int32_t, "fam_drop", Fcap);
    if (Fcap > 0 && !drop_zeroed) HIPCHK(hipMemsetAsync(fam_drop, 0, sizeof(int32_t) * Fcap, ctx->stream));
    RC(scan_emit(ctx, g, segf, R, &F, "scan_fam", EmitFamStarts{validf, fam_beg, fam_drop, d_ndrop, Fcap, ctx->d_err}));
    g.F = F;
    fam_beg = GB(int32_t, "fam_beg", F);
    int32_t* fam_end = GB(int32_t, "fam_end", F);
    int32_t* fam_n = GB(int32_t, "fam_n", F);
    int32_t* fam_first = GB(int32_t, "fam_first", F);
    int32_t* fam_region = GB(int32_t, "fam_region", F);
    uint64_t* fam_hash = GB(uint64_t, "fam_hash", F);
    int32_t* cfam = GB(int32_t, "cfam", R);
    int32_t* fam_o = GB(int32_t, "fam_o", F);
    // the passes whose stage joins the grouping (DCS, SC: no bad-read list) build the family tags
    // here; the SSCS pass never joins
    g.fam_tags_built = false;
    TagKey* fam_tag = nullptr;
    int32_t* fam_rec = nullptr;
    if (!g.badread) {
        fam_tag = GB(TagKey, "fam_tag", F);
        fam_rec = GB(int32_t, "fam_rec", F);
    }
    if (F > 0) {
        ProfScope ps(ctx, "k_fam_build");
        hipLaunchKernelGGL(k_fam_build, dim3(nblk(F)), dim3(256), 0, ctx->stream, F, R, fam_beg, fam_drop,
                           rs_val, rs_key, pr_region, (const uint64_t*)(g.coord_sorted ? g.buf["rec_thash"].p : nullptr),
                           (const int32_t*)mem_rec, fam_end, fam_n, fam_first, fam_region, fam_hash, cflag,
                           cfam, fam_o, PV, T, fam_tag, fam_rec);
    }
    g.fam_tags_built = fam_tag != nullptr;
    RC(planned_total(ctx, g, "n_drop", d_ndrop, &V));
    V = R - V;   // members kept
    // ---- 5. tag_dict insertion order (family creation order)
    int64_t F2 = 0;
    int32_t* fam_by_k = GB(int32_t, "fam_by_k", F);
    int32_t* fam_k = GB(int32_t, "fam_k", F);
    int32_t* pair_by_k = GB(int32_t, "pair_by_k", F);
    int32_t* fsz = GB(int32_t, "fam_sizes_by_creation", F);
    RC(scan_emit(ctx, g, cflag, R, &F2, "scan_creation", EmitCreation{cfam, fam_n, fam_by_k, fam_k, pair_by_k, fsz}));
    // ---- 6. csn_pair_dict: group creation events by consensus tag
    uint32_t* csegf = GB(uint32_t, "csegf", F);
    uint8_t* emark = GB(uint8_t, "emark", (F + 15) & ~15LL);
    int32_t* e1k = GB(int32_t, "e1k", F);
    bool fast_ok = false;
    if (F > 0) {
        // with the stream in table order (each record once) the global table takes the pairs with an
        // end in a deep group (at most the deep read ends); otherwise every entry
        const bool tiles = g.coord_sorted && g.ident && bigE;
        uint64_t size = 1024;
        while (size < (uint64_t)(tiles ? 2 * n_deep : 2 * F)) size <<= 1;
        unsigned long long* cht = GB(unsigned long long, "csn_ht_key", (int64_t)size);
        uint32_t* shared = plan_slot(ctx, g, "csn_shared", &brc);
        if (brc) return brc;
        RC(fill.add(cht, sizeof(unsigned long long) * size, ~0u));
        RC(fill.add(shared, 4, 0u));
        RC(fill.launch());
        {
            ProfScope ps(ctx, "k_csn_fast");
            hipLaunchKernelGGL(k_csn_fast, dim3((unsigned)((F + CT - 1) / CT)), dim3(256), 0, ctx->stream, F, pair_by_k,
                               chash, tiles ? (const uint32_t*)bigE : (const uint32_t*)nullptr,
                               cht, size - 1, emark, e1k, shared);
        }
        int64_t sh = 0;
        RC(planned_total(ctx, g, "csn_shared", shared, &sh));
        fast_ok = sh == 0;
    }
    if (F > 0 && !fast_ok) {
        uint64_t* ekey = GB(uint64_t, "ekey", F);
        uint32_t* eval = GB(uint32_t, "eval", F);
        uint64_t* es_key = GB(uint64_t, "es_key", F);
        uint32_t* es_val = GB(uint32_t, "es_val", F);
        hipLaunchKernelGGL(k_csn_keys, dim3(nblk(F)), dim3(256), 0, ctx->stream, F, fam_by_k, fam_first, chash, ekey, eval);
        RC(sort_pairs(ctx, ekey, es_key, eval, es_val, F, "sort_csn"));
        HIPCHK(hipMemsetAsync(emark, 0, std::max<int64_t>(F, 1), ctx->stream));
        ProfScope ps(ctx, "k_csn");
        hipLaunchKernelGGL(k_csn_mark, dim3(nblk(F)), dim3(256), 0, ctx->stream, F, es_key, es_val, fam_by_k,
                           fam_first, PV, T, csegf, ctx->d_err);
        hipLaunchKernelGGL(k_csn_entries, dim3(nblk(F)), dim3(256), 0, ctx->stream, F, csegf, es_val, fam_by_k,
                           fam_region, emark, e1k, ctx->d_err, ctx->d_cnt);
    }
    g.csn_fast = fast_ok;
    int64_t E = 0;
    int32_t* ent_f = GB(int32_t, "ent_f", 2 * F);   // capacity; sized E below
    int32_t* ent_pair = GB(int32_t, "ent_pair", F);
    uint8_t* has2 = GB(uint8_t, "has2", (F + 15) & ~15LL);   // byte flags (16-B padded for the scan)
    RC(scan_emit(ctx, g, emark, F, &E, "scan_entries",
                 EmitEntries{e1k, fam_by_k, pair_by_k, ent_f, ent_pair, fam_o, has2}));
    g.E = E;
    ent_f = GB(int32_t, "ent_f", 2 * E);
    ent_pair = GB(int32_t, "ent_pair", E);
    if (g.overlap && E > 0)
        hipLaunchKernelGGL(k_overlap_keyerror, dim3(nblk(E)), dim3(256), 0, ctx->stream, E, (const int32_t*)ent_f,
                           (const int32_t*)fam_beg, (const int32_t*)fam_end, (const int32_t*)fam_region,
                           (const uint32_t*)rs_val, (const int32_t*)pr_region, ctx->d_err);
    // ---- counters + error word
    uint32_t bits = 0;
    bool plan_ok = true;
    RC(finish_pass(ctx, g, &bits, true, &plan_ok));
    if (bits & EB_NEEDSORT) return CC_E_NEEDSORT;   // before the plan check: the re-run is exact
    if (bits & EB_DEEPSORT) return CC_E_DEEPSORT;
    if (!plan_ok) return CC_E_PLAN;
    g.counters[CC_CNT_COUNTER] = S - g.counters[CC_CNT_FOREIGN] - g.counters[CC_CNT_UNMAPPED];
    g.counters[CC_CNT_PAIRS] = P;
    g.counters[CC_CNT_READ_ENDS] = R;
    g.counters[CC_CNT_FAMILIES] = F;
    g.counters[CC_CNT_ENTRIES] = E;
    g.counters[CC_CNT_DROPPED] = R - V;
    g.members_built = members;
    return err_code(ctx, bits);
}

int read_bam_run(cc_ctx* ctx, int32_t gid) {
    Group& g = *ctx->groups[gid];
    int rc = run_planned(ctx, g, "read_bam", [&] { return read_bam_pass(ctx, gid); });
    for (int k = 0; k < 2 && (rc == CC_E_NEEDSORT || rc == CC_E_DEEPSORT); ++k) {
        // a qname seen more than twice: pair_dict's stream order needs the sort path; a long deep
        // family out of end order: the deep ends take the sorted path (both from now on)
        if (rc == CC_E_NEEDSORT) g.force_sort = true;
        else g.no_deep_fam = true;
        g.planned["read_bam"] = false;
        rc = run_planned(ctx, g, "read_bam", [&] { return read_bam_pass(ctx, gid); });
    }
    return rc;
}

}  // namespace

extern "C" {

int cc_read_bam(cc_ctx* ctx, int32_t table_id, int64_t S, const int32_t* stream_rec, const int32_t* stream_region,
                int32_t n_regions, const int32_t* region_run, const cc_read_bam_params* prm, int32_t* group_id) {
    if (!ctx || !prm || !group_id || !ctx->tables.count(table_id) || S < 0 || S >= INT32_MAX / 2) return CC_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    int32_t gid = ctx->next_id++;
    ctx->groups[gid].reset(new Group());
    Group& g = *ctx->groups[gid];
    g.table = table_id;
    g.seed = prm->seed;
    g.scoped = prm->scope_by_run;
    g.delim_filter = prm->delim_filter;
    g.badread = prm->badread_file;
    g.coord_sorted = prm->coord_sorted;
    g.S = S;
    g.ident = S == ctx->tables[table_id].n;
    for (int64_t i = 0; g.ident && i < S; ++i) g.ident = stream_rec[i] == (int32_t)i;
    if (!g.ident) {   // a record in two stream entries: overlapping bed regions
        std::vector<bool> seen((size_t)ctx->tables[table_id].n, false);
        for (int64_t i = 0; i < S && !g.overlap; ++i) {
            const int32_t r = stream_rec[i];
            if (r < 0 || r >= ctx->tables[table_id].n) continue;
            g.overlap = seen[(size_t)r];
            seen[(size_t)r] = true;
        }
        // a record with two stream entries can complete two pairs: the record-indexed paths of a
        // sorted table (one read end per record) do not apply, the stream-indexed sort path does
        if (g.overlap) g.coord_sorted = 0;
    }
    int brc = 0;
    int32_t* d_srec = GB(int32_t, "stream_rec", S);
    int32_t* d_sreg = GB(int32_t, "stream_region", S);
    int32_t* d_run = GB(int32_t, "region_run", std::max<int32_t>(n_regions, 1));
    if (S > 0) {
        HIPCHK(hipMemcpyAsync(d_srec, stream_rec, sizeof(int32_t) * S, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(d_sreg, stream_region, sizeof(int32_t) * S, hipMemcpyHostToDevice, ctx->stream));
    }
    if (n_regions > 0)
        HIPCHK(hipMemcpyAsync(d_run, region_run, sizeof(int32_t) * n_regions, hipMemcpyHostToDevice, ctx->stream));
    *group_id = gid;
    return read_bam_run(ctx, gid);
}

// Re-run read_bam on a group whose stream is already resident (bench steps), with a new seed.
int cc_read_bam_rerun(cc_ctx* ctx, int32_t group_id, uint64_t seed) {
    if (!ctx || !ctx->groups.count(group_id)) return CC_E_INVALID;
    ctx->groups[group_id]->seed = seed;
    return read_bam_run(ctx, group_id);
}

int cc_group_counters(cc_ctx* ctx, int32_t group_id, int64_t* counters) {
    if (!ctx || !ctx->groups.count(group_id) || !counters) return CC_E_INVALID;
    memcpy(counters, ctx->groups[group_id]->counters, sizeof(int64_t) * CC_NUM_COUNTERS);
    return 0;
}

int cc_group_free(cc_ctx* ctx, int32_t group_id) {
    if (!ctx || !ctx->groups.count(group_id)) return CC_E_INVALID;
    (void)hipStreamSynchronize(ctx->stream);
    {
        Group* gp = ctx->groups[group_id].get();
        std::vector<DeferredCheck> keep;
        for (auto& d : ctx->deferred)
            if (d.g != gp) keep.push_back(d);
        ctx->deferred.swap(keep);
    }
    for (auto& b : ctx->groups[group_id]->buf)
        if (b.second.p) (void)hipFree(b.second.p);
    ctx->groups.erase(group_id);
    return 0;
}

// SSCS region loop (SSCS_maker.py:312-339): every csn entry with two tags emits
// both families; size 1 -> singleton record renamed, else consensus_maker.
int cc_consensus_maker(cc_ctx* ctx, int32_t group_id, double cutoff, int64_t* n_out) {
    if (!ctx || !ctx->groups.count(group_id)) return CC_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    Group& g = *ctx->groups[group_id];
    auto pass = [&]() -> int {
        const DevTable& T = ctx->tables[g.table];
        int brc = 0;
        const int64_t E = g.E, F = g.F, R = g.R;
        if (!g.members_built) {   // a pass that did not write the member records (see read_bam_pass)
            uint4* mm = GB(uint4, "mem_meta", R);
            if (R > 0)
                hipLaunchKernelGGL(k_mem_meta, dim3(nblk(R)), dim3(256), 0, ctx->stream, R,
                                   (const int32_t*)g.buf["mem_rec"].p, (const uint32_t*)g.buf["mem_valid"].p, T, mm);
            g.members_built = true;
        }
        const uint8_t* has2 = (const uint8_t*)g.buf["has2"].p;   // by the pass's entry scan (EmitEntries)
        uint32_t* hx = GB(uint32_t, "hx", (E + 3) & ~3LL);
        int64_t E2 = 0;
        RC(scan_total(ctx, g, has2, hx, E, &E2, "scan_emit"));
        const int64_t NE = 2 * E2;
        int32_t* emit_fam = GB(int32_t, "emit_fam", NE);
        int32_t* emit_n = GB(int32_t, "emit_n", NE);
        int32_t* emit_rec = GB(int32_t, "emit_rec", NE);
        int32_t* emit_ckey = GB(int32_t, "emit_ckey", 9 * E2);   // per emitted entry (both its records)
        uint8_t* needv = GB(uint8_t, "needv", (NE + 15) & ~15LL);   // byte flags (16-B padded for the scan)
        int2* emit_span = GB(int2, "emit_span", NE);
        uint32_t* vxs = GB(uint32_t, "vxs", (NE + 3) & ~3LL);
        if (E > 0) {
            ProfScope ps(ctx, "k_sscs_emit");
            hipLaunchKernelGGL(k_sscs_emit, dim3(nblk(E)), dim3(256), 0, ctx->stream, E, (const int32_t*)g.buf["ent_f"].p,
                               (const int32_t*)g.buf["ent_pair"].p, has2, hx, (const int32_t*)g.buf["fam_n"].p,
                               (const int32_t*)g.buf["fam_beg"].p, (const int32_t*)g.buf["fam_end"].p,
                               (const int32_t*)g.buf["mem_rec"].p, emit_fam, emit_n, emit_rec, needv, emit_span,
                               pair_view(g), T, emit_ckey);
        }
        int64_t NV = 0;
        RC(vote_families(ctx, g, T, NE, needv, vxs, emit_fam, emit_span, cutoff, &NV));
        // badReads list + read_families sizes (host formats the text)
        const int64_t S = g.S;
        int64_t NB = 0;
        int32_t* bad_rec = GB(int32_t, "bad_rec", S);   // capacity; sized NB below
        // the flagged entries are counted by read_bam (its counters are on the host): none, no scan
        if (g.counters[CC_CNT_BAD_LISTED] > 0)
            RC(scan_emit(ctx, g, (const uint8_t*)g.buf["badflag"].p, S, &NB, "scan_bad",
                         EmitGather{(const int32_t*)g.buf["stream_rec"].p, bad_rec}));
        bad_rec = GB(int32_t, "bad_rec", NB);
        // (fam_sizes_by_creation: written by the pass's creation scan, EmitCreation)
        (void)F;
        (void)R;
        uint32_t bits = 0;
        bool plan_ok = true;
        RC(finish_pass(ctx, g, &bits, false, &plan_ok));
        if (!plan_ok) return CC_E_PLAN;
        if (n_out) *n_out = NE;
        return err_code(ctx, bits);
    };
    return run_planned(ctx, g, "sscs", pass);
}

int cc_duplex_consensus(cc_ctx* ctx, int32_t group_id, const int32_t* bc_swap, int32_t n_bc, int64_t* n_out) {
    if (!ctx || !ctx->groups.count(group_id) || (!bc_swap && n_bc > 0)) return CC_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    Group& g = *ctx->groups[group_id];
    auto pass = [&]() -> int {
        const DevTable& T = ctx->tables[g.table];
        int brc = 0;
        const int64_t Q = 2 * g.E;
        g.Q = Q;
        HIPCHK(hipMemsetAsync(ctx->d_err, 0, 4, ctx->stream));
        int32_t* d_swap = GB(int32_t, "bc_swap", std::max(n_bc, 1));
        RC(upload_swap(ctx, g, d_swap, bc_swap, n_bc));
        int32_t* dec = GB(int32_t, "dec", Q);
        int32_t* t_rec = GB(int32_t, "t_rec", Q);
        int32_t* p_rec = GB(int32_t, "p_rec", Q);
        uint8_t* fl_dcs = GB(uint8_t, "fl_dcs", (Q + 15) & ~15LL);   // byte flags (16-B padded for the scan)
        if (!g.local_groups) RC(build_ht(ctx, g));   // duplex partners are found among position-group neighbours
        RC(ensure_fam_tags(ctx, g));
        GroupView G = view_of(g);
        if (Q > 0) {
            ProfScope ps(ctx, "k_dcs_decide");
            hipLaunchKernelGGL(k_dcs_decide, dim3(nblk(Q)), dim3(256), 0, ctx->stream, Q, G, d_swap, n_bc, dec, t_rec,
                               p_rec, fl_dcs, ctx->d_err);
        }
        int64_t NV = 0;
        int32_t* vslot = GB(int32_t, "vslot", Q);
        int4* vpair = GB(int4, "vpair", Q);   // capacity; sized NV below
        RC(scan_emit(ctx, g, (const uint8_t*)fl_dcs, Q, &NV, "scan_dcs", EmitVotePairs{t_rec, p_rec, dec, vslot, vpair}));
        g.NV = NV;
        const int32_t qstride = (int32_t)((T.max_len + 15) & ~15);
        uint8_t* cons_seq = GB(uint8_t, "cons_seq", NV * (qstride / 2));
        uint8_t* cons_qual = GB(uint8_t, "cons_qual", NV * qstride);
        int32_t* vmeta = GB(int32_t, "vote_meta", 5 * NV);
        if (NV > 0) {
            ProfScope ps(ctx, "k_duplex_vote_dcs");
            const int32_t chunks = std::min(64, std::max(1, (T.max_len + SV_POS - 1) / SV_POS));   // lanes per output
            const int32_t fpw = 64 / chunks;
            hipLaunchKernelGGL(k_duplex_vote_swar, dim3(nblk((NV + fpw - 1) / fpw, 4)), dim3(256), 0, ctx->stream, NV, 0,
                               fpw, chunks, (const int4*)vpair, T, T, qstride, cons_seq, cons_qual, vmeta, ctx->d_err);
        }
        uint32_t bits = 0;
        bool plan_ok = true;
        RC(finish_pass(ctx, g, &bits, false, &plan_ok));
        if (!plan_ok) return CC_E_PLAN;
        if (n_out) *n_out = Q;
        return err_code(ctx, bits);
    };
    return run_planned(ctx, g, "dcs", pass);
}

int cc_singleton_correction(cc_ctx* ctx, int32_t sgroup, int32_t ssgroup, const int32_t* bc_swap, int32_t n_bc,
                            int64_t* n_out) {
    if (!ctx || !ctx->groups.count(sgroup) || !ctx->groups.count(ssgroup) || (!bc_swap && n_bc > 0))
        return CC_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    Group& g = *ctx->groups[sgroup];
    Group& s = *ctx->groups[ssgroup];
    auto pass = [&]() -> int {
        const DevTable& TA = ctx->tables[g.table];
        const DevTable& TB = ctx->tables[s.table];
        int brc = 0;
        const int64_t Q = 2 * g.E;
        g.Q = Q;
        HIPCHK(hipMemsetAsync(ctx->d_err, 0, 4, ctx->stream));
        int32_t* d_swap = GB(int32_t, "bc_swap", std::max(n_bc, 1));
        RC(upload_swap(ctx, g, d_swap, bc_swap, n_bc));
        int32_t* dec = GB(int32_t, "dec", Q);
        int32_t* t_rec = GB(int32_t, "t_rec", Q);
        int32_t* p_rec = GB(int32_t, "p_rec", Q);
        uint8_t* fl = GB(uint8_t, "fl_corr", (Q + 15) & ~15LL);   // byte flags (16-B padded for the scan)
        if (!g.local_groups) RC(build_ht(ctx, g));
        RC(ensure_fam_tags(ctx, g));
        RC(ensure_fam_tags(ctx, s));
        GroupView G = view_of(g), SV = view_of(s);
        // the SSCS side is another table: its families by position bucket, else hashed lookups
        bool sb = false;
        RC(build_fam_buckets(ctx, s, &SV, &sb));
        if (!sb) {
            RC(build_ht(ctx, s));
            SV = view_of(s);
        }
        if (Q > 0) {
            ProfScope ps(ctx, "k_sc_decide");
            hipLaunchKernelGGL(k_sc_decide, dim3(nblk(Q)), dim3(256), 0, ctx->stream, Q, G, SV,
                               (const int32_t*)g.buf["region_run"].p, d_swap, n_bc, dec, t_rec, p_rec, fl, ctx->d_err);
        }
        int64_t NV = 0;
        int32_t* vslot = GB(int32_t, "vslot", Q);
        int4* vpair = GB(int4, "vpair", Q);   // capacity; sized NV below
        RC(scan_emit(ctx, g, (const uint8_t*)fl, Q, &NV, "scan_sc", EmitVotePairs{t_rec, p_rec, dec, vslot, vpair}));
        g.NV = NV;
        const int32_t ml = std::max(TA.max_len, TB.max_len);
        const int32_t qstride = (int32_t)((ml + 15) & ~15);
        uint8_t* cons_seq = GB(uint8_t, "cons_seq", NV * (qstride / 2));
        uint8_t* cons_qual = GB(uint8_t, "cons_qual", NV * qstride);
        int32_t* vmeta = GB(int32_t, "vote_meta", 5 * NV);
        if (NV > 0) {
            ProfScope ps(ctx, "k_duplex_vote_sc");
            const int32_t chunks = std::min(64, std::max(1, (ml + SV_POS - 1) / SV_POS));   // lanes per output
            const int32_t fpw = 64 / chunks;
            hipLaunchKernelGGL(k_duplex_vote_swar, dim3(nblk((NV + fpw - 1) / fpw, 4)), dim3(256), 0, ctx->stream, NV, 1,
                               fpw, chunks, (const int4*)vpair, TA, TB, qstride, cons_seq, cons_qual, vmeta, ctx->d_err);
        }
        // names: consensus tag of the singleton entry + ':1' (singleton_correction.py:286)
        int32_t* q_pair = GB(int32_t, "q_pair", Q);
        int32_t* q_ckey = GB(int32_t, "q_ckey", 9 * Q);
        if (Q > 0) {
            hipLaunchKernelGGL(k_q_pairs, dim3(nblk(Q)), dim3(256), 0, ctx->stream, Q, (const int32_t*)g.buf["ent_pair"].p,
                               q_pair);
            hipLaunchKernelGGL(k_ckey_out, dim3(nblk(Q)), dim3(256), 0, ctx->stream, Q, q_pair, pair_view(g),
                               ctx->tables[g.table], q_ckey);
        }
        uint32_t bits = 0;
        bool plan_ok = true;
        RC(finish_pass(ctx, g, &bits, false, &plan_ok));
        if (!plan_ok) return CC_E_PLAN;
        if (n_out) *n_out = Q;
        return err_code(ctx, bits);
    };
    return run_planned(ctx, g, "sc", pass);
}

int64_t cc_fetch(cc_ctx* ctx, int32_t group_id, const char* name, void* dst, int64_t cap) {
    if (!ctx || !ctx->groups.count(group_id) || !name) return CC_E_INVALID;
    Group& g = *ctx->groups[group_id];
    auto it = g.buf.find(name);
    if (it == g.buf.end()) {
        ctx->err = std::string("no result array named ") + name;
        return CC_E_INVALID;
    }
    int64_t bytes = (int64_t)it->second.used;
    if (!dst) return bytes;
    int64_t nb = std::min(bytes, cap);
    if (nb > 0) {
        HIPCHK(hipMemcpyAsync(dst, it->second.p, (size_t)nb, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
    }
    return nb;
}


// ------------------------------------------------------------------ function-level boundary
// consensus_maker / duplex_consensus on caller-given reads: the reads are
// records of an uploaded table, the families (or pairs) are given by record index.  The same
// kernels as the stage calls run them on the member records built at upload (k_table_cols); the
// table's column error bits go into the call's word first.
}  // extern "C"

namespace {
int function_prep(cc_ctx* ctx, const DevTable& T) {
    if (T.n > 0) {
        ProfScope ps(ctx, "k_build_meta");
        hipLaunchKernelGGL(k_build_meta, dim3(1), dim3(BC_T), 0, ctx->stream, T, (int32_t*)nullptr, ctx->d_err,
                           (int32_t*)nullptr, (uint32_t*)nullptr, (int64_t)0);   // the table's error bits
    }
    return 0;
}

Group& scratch_group(cc_ctx* ctx, int32_t table) {
    if (!ctx->scratch) ctx->scratch.reset(new Group());
    Group& g = *ctx->scratch;
    g.table = table;
    g.fast = false;
    g.verify.clear();
    return g;
}

// result rows of stride `from` (device) to caller rows of stride `to` (host)
int copy_rows(cc_ctx* ctx, void* dst, int64_t to, const void* src, int64_t from, int64_t width, int64_t rows) {
    if (rows <= 0 || width <= 0) return 0;
    HIPCHK(hipMemcpy2DAsync(dst, (size_t)to, src, (size_t)from, (size_t)width, (size_t)rows, hipMemcpyDeviceToHost,
                            ctx->stream));
    return 0;
}
}  // namespace

extern "C" {

int cc_sscs_vote(cc_ctx* ctx, int32_t table_id, const int32_t* member_index, const int64_t* fam_offsets, int64_t nfam,
                 double cutoff, uint8_t* out_seq, uint8_t* out_qual, int32_t* out_meta, int32_t out_stride) {
    if (!ctx || !ctx->tables.count(table_id) || nfam < 0 || (nfam > 0 && (!fam_offsets || !out_seq || !out_qual ||
                                                                         !out_meta)))
        return CC_E_INVALID;
    if (nfam > 0 && fam_offsets[nfam] > 0 && !member_index) return CC_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    const DevTable T = ctx->tables[table_id];
    if (out_stride < T.max_len || (out_stride & 1)) {
        ctx->err = "out_stride must be even and at least the table's longest read";
        return CC_E_INVALID;
    }
    const int64_t R = nfam > 0 ? fam_offsets[nfam] : 0;
    if (nfam > 0 && fam_offsets[0] != 0) { ctx->err = "fam_offsets[0] must be 0"; return CC_E_INVALID; }
    if (R > INT32_MAX) { ctx->err = "too many members"; return CC_E_INVALID; }
    std::vector<int32_t> beg(nfam), end(nfam), cnt(nfam), fam(nfam);
    std::vector<int2> span(nfam);
    for (int64_t k = 0; k < nfam; ++k) {
        if (fam_offsets[k + 1] <= fam_offsets[k]) {
            // consensus_maker(readList) reads readList[0] (SSCS_maker.py:107): an empty family raises
            ctx->err = "IndexError: empty family (SSCS_maker.py:107)";
            return CC_E_INVALID;
        }
        beg[k] = (int32_t)fam_offsets[k];
        end[k] = (int32_t)fam_offsets[k + 1];
        cnt[k] = end[k] - beg[k];
        fam[k] = (int32_t)k;
        span[k] = make_int2(beg[k], cnt[k]);
    }
    for (int64_t j = 0; j < R; ++j)
        if (member_index[j] < 0 || member_index[j] >= T.n) { ctx->err = "member index outside the table"; return CC_E_INVALID; }
    Group& g = scratch_group(ctx, table_id);
    int brc = 0;
    int32_t* mem_rec = GB(int32_t, "mem_rec", R);
    uint32_t* mem_valid = GB(uint32_t, "mem_valid", R);
    uint4* mem_meta = GB(uint4, "mem_meta", R);
    int32_t* d_beg = GB(int32_t, "fam_beg", nfam);
    int32_t* d_end = GB(int32_t, "fam_end", nfam);
    int32_t* d_n = GB(int32_t, "fam_n", nfam);
    int32_t* d_fam = GB(int32_t, "emit_fam", nfam);
    int2* d_span = GB(int2, "emit_span", nfam);
    uint8_t* needv = GB(uint8_t, "needv", (nfam + 15) & ~15LL);
    uint32_t* vxs = GB(uint32_t, "vxs", nfam);
    if (R > 0) HIPCHK(hipMemcpyAsync(mem_rec, member_index, sizeof(int32_t) * R, hipMemcpyHostToDevice, ctx->stream));
    if (nfam > 0) {
        HIPCHK(hipMemcpyAsync(d_beg, beg.data(), sizeof(int32_t) * nfam, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(d_end, end.data(), sizeof(int32_t) * nfam, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(d_n, cnt.data(), sizeof(int32_t) * nfam, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(d_fam, fam.data(), sizeof(int32_t) * nfam, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(d_span, span.data(), sizeof(int2) * nfam, hipMemcpyHostToDevice, ctx->stream));
    }
    {
        Fills fill(ctx);
        RC(fill.add(mem_valid, sizeof(uint32_t) * R, 1u));
        RC(fill.add(needv, (size_t)((nfam + 15) & ~15LL), 0x01010101u));
        RC(fill.add(ctx->d_err, 64, 0u));
        RC(fill.launch());
    }
    RC(function_prep(ctx, T));
    if (R > 0)
        hipLaunchKernelGGL(k_mem_meta, dim3(nblk(R)), dim3(256), 0, ctx->stream, R, (const int32_t*)mem_rec,
                           (const uint32_t*)mem_valid, T, mem_meta);
    int64_t NV = 0;
    RC(vote_families(ctx, g, T, nfam, needv, vxs, d_fam, d_span, cutoff, &NV));
    uint32_t bits = 0;
    RC(read_err(ctx, &bits));   // synchronises: the caller's arrays were read
    if (bits) return err_code(ctx, bits);
    // every family voted and the vote slots are 0..nfam-1 in family order (needv all set)
    const int64_t qstride = (T.max_len + 15) & ~15;
    RC(copy_rows(ctx, out_qual, out_stride, g.buf["cons_qual"].p, qstride, T.max_len, NV));
    RC(copy_rows(ctx, out_seq, out_stride / 2, g.buf["cons_seq"].p, qstride / 2, (T.max_len + 1) / 2, NV));
    if (NV > 0)
        HIPCHK(hipMemcpyAsync(out_meta, g.buf["vote_meta"].p, sizeof(int32_t) * 5 * NV, hipMemcpyDeviceToHost,
                              ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return 0;
}

int cc_pair_vote(cc_ctx* ctx, int32_t mode, int32_t table_a, int32_t table_b, const int32_t* rec_a, const int32_t* rec_b,
                 int64_t n, uint8_t* out_seq, uint8_t* out_qual, int32_t* out_meta, int32_t out_stride) {
    if (!ctx || !ctx->tables.count(table_a) || !ctx->tables.count(table_b) || (mode != 0 && mode != 1) || n < 0 ||
        (n > 0 && (!rec_a || !rec_b || !out_seq || !out_qual || !out_meta)))
        return CC_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    const DevTable TA = ctx->tables[table_a], TB = ctx->tables[table_b];
    const int32_t ml = std::max(TA.max_len, TB.max_len);
    if (out_stride < ml || (out_stride & 1)) {
        ctx->err = "out_stride must be even and at least the tables' longest read";
        return CC_E_INVALID;
    }
    if (n > INT32_MAX) return CC_E_INVALID;
    for (int64_t i = 0; i < n; ++i)
        if (rec_a[i] < 0 || rec_a[i] >= TA.n || rec_b[i] < 0 || rec_b[i] >= TB.n) {
            ctx->err = "record index outside its table";
            return CC_E_INVALID;
        }
    Group& g = scratch_group(ctx, table_a);
    int brc = 0;
    int4* vpair = GB(int4, "vpair", n);
    const int32_t qstride = (int32_t)((ml + 15) & ~15);
    uint8_t* cons_seq = GB(uint8_t, "cons_seq", n * (qstride / 2));
    uint8_t* cons_qual = GB(uint8_t, "cons_qual", n * qstride);
    int32_t* vmeta = GB(int32_t, "vote_meta", 5 * n);
    if (n > 0) {
        // {read1, read2, decision 0 (read2 in table_b), entry}
        std::vector<int4> vp((size_t)n);
        for (int64_t i = 0; i < n; ++i) vp[i] = make_int4(rec_a[i], rec_b[i], 0, (int32_t)i);
        HIPCHK(hipMemcpyAsync(vpair, vp.data(), sizeof(int4) * n, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));   // vp is a local
    }
    {
        Fills fill(ctx);
        RC(fill.add(ctx->d_err, 64, 0u));
        RC(fill.launch());
    }
    RC(function_prep(ctx, TA));
    if (table_b != table_a) RC(function_prep(ctx, TB));
    if (n > 0) {
        ProfScope ps(ctx, mode ? "k_duplex_vote_sc" : "k_duplex_vote_dcs");
        const int32_t chunks = std::min(64, std::max(1, (ml + SV_POS - 1) / SV_POS));
        const int32_t fpw = 64 / chunks;
        hipLaunchKernelGGL(k_duplex_vote_swar, dim3(nblk((n + fpw - 1) / fpw, 4)), dim3(256), 0, ctx->stream, n, mode,
                           fpw, chunks, (const int4*)vpair, TA, TB, qstride, cons_seq, cons_qual, vmeta, ctx->d_err);
    }
    uint32_t bits = 0;
    RC(read_err(ctx, &bits));
    if (bits) return err_code(ctx, bits);
    RC(copy_rows(ctx, out_qual, out_stride, cons_qual, qstride, ml, n));
    RC(copy_rows(ctx, out_seq, out_stride / 2, cons_seq, qstride / 2, (ml + 1) / 2, n));
    if (n > 0)
        HIPCHK(hipMemcpyAsync(out_meta, vmeta, sizeof(int32_t) * 5 * n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return 0;
}

}  // extern "C"

// ---- grouping and duplex joins on caller-given keys ---------------
// Keys are opaque fixed-width byte strings (key_bytes a multiple of 4): the caller's packed tags.
// Equality is exact (word compare); the 64-bit hashes only place keys in an open-addressing table
// whose slots hold the index of the first key inserted there (atomicCAS), so every key finds the
// slot of its class in one probe sequence.
namespace {
constexpr int KEY_MAX_WORDS = 64;   // key_bytes <= 256

__device__ __forceinline__ uint64_t key_hash(const uint32_t* __restrict__ k, int kw, uint64_t seed) {
    uint64_t h = seed ^ (uint64_t)kw;
    int w = 0;
    for (; w + 1 < kw; w += 2) h = hcomb(h, (uint64_t)k[w] | ((uint64_t)k[w + 1] << 32));
    if (w < kw) h = hcomb(h, (uint64_t)k[w]);
    return h;
}
__device__ __forceinline__ bool key_eq(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, int kw) {
    for (int w = 0; w < kw; ++w)
        if (a[w] != b[w]) return false;
    return true;
}

// key i enters the table (slot -> first key index there); *slot_of = its class's slot.  dup: a key
// equal to one inserted before is reported (cc_duplex_join needs unique keys).
__global__ __launch_bounds__(256) void k_key_insert(int64_t n, const uint32_t* __restrict__ keys, int kw, uint64_t seed,
                                                    int32_t* __restrict__ slot_key, uint64_t mask,
                                                    int32_t* __restrict__ slot_of, int32_t* __restrict__ slot_first,
                                                    int32_t* __restrict__ slot_cnt, uint32_t* __restrict__ dup) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* k = keys + i * (int64_t)kw;
    uint64_t s = key_hash(k, kw, seed) & mask;
    for (uint64_t probe = 0; probe <= mask; ++probe) {
        const int32_t prev = atomicCAS(&slot_key[s], -1, (int32_t)i);
        if (prev == -1 || key_eq(keys + (int64_t)prev * kw, k, kw)) {
            if (prev != -1 && dup) atomicOr(dup, 1u);
            if (slot_of) slot_of[i] = (int32_t)s;
            if (slot_first) atomicMin(&slot_first[s], (int32_t)i);
            if (slot_cnt) atomicAdd(&slot_cnt[s], 1);
            return;
        }
        s = (s + 1) & mask;
    }
}

// the index of the key equal to probe key i among the inserted keys (-1: none)
__global__ __launch_bounds__(256) void k_key_probe(int64_t n, const uint32_t* __restrict__ probes,
                                                   const uint32_t* __restrict__ keys, int kw, uint64_t seed,
                                                   const int32_t* __restrict__ slot_key, uint64_t mask,
                                                   int32_t* __restrict__ out, int32_t* __restrict__ first_of,
                                                   int32_t* __restrict__ indeg) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* k = probes + i * (int64_t)kw;
    uint64_t s = key_hash(k, kw, seed) & mask;
    int32_t found = -1;
    for (uint64_t probe = 0; probe <= mask; ++probe) {
        const int32_t j = slot_key[s];
        if (j == -1) break;
        if (key_eq(keys + (int64_t)j * kw, k, kw)) { found = j; break; }
        s = (s + 1) & mask;
    }
    out[i] = found;
    if (found >= 0 && first_of) atomicMin(&first_of[found], (int32_t)i);   // SC: the first singleton per SSCS
    if (found >= 0 && indeg) atomicAdd(&indeg[found], 1);
}

// cc_group: a key starts its family at its class's first index
__global__ __launch_bounds__(256) void k_group_starts(int64_t n, const int32_t* __restrict__ slot_of,
                                                      const int32_t* __restrict__ slot_first, uint32_t* __restrict__ start) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) start[i] = slot_first[slot_of[i]] == (int32_t)i ? 1u : 0u;
}
// per family (in first-seen order) its size; per key its family number as the sort key
__global__ __launch_bounds__(256) void k_group_fams(int64_t n, const int32_t* __restrict__ slot_of,
                                                    const int32_t* __restrict__ slot_first,
                                                    const int32_t* __restrict__ slot_cnt, const uint32_t* __restrict__ fx,
                                                    uint32_t* __restrict__ fam_size, uint64_t* __restrict__ fkey,
                                                    uint32_t* __restrict__ fval) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t s = slot_of[i], f0 = slot_first[s];
    const uint32_t fam = fx[f0];
    if (f0 == (int32_t)i) fam_size[fam] = (uint32_t)slot_cnt[s];
    fkey[i] = fam;
    fval[i] = (uint32_t)i;
}

// cc_duplex_join decisions with every entry's partner resolved to an index (p: among the entries,
// xs: among the SSCS keys, SC only), processing order = entry index.  The chain walks of k_dcs_decide
// / k_sc_decide; *seq set when a chain is longer than DUPLEX_CHAIN or (SC) two entries share a
// singleton partner, whose deletions the chain walk does not see: then k_join_serial decides.
__global__ __launch_bounds__(256) void k_join_decide(int64_t n, int mode, const int32_t* __restrict__ p,
                                                     const int32_t* __restrict__ xs, const int32_t* __restrict__ xfirst,
                                                     const int32_t* __restrict__ indeg, int32_t* __restrict__ dec,
                                                     int32_t* __restrict__ part, uint32_t* __restrict__ seq,
                                                     uint32_t* __restrict__ err) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t d = 0, pr = -1;
    if (mode == 0) {
        int32_t x = (int32_t)i, g = -1;
        int nc = 0;
        bool present = false;
        while (true) {
            g = p[x];
            present = g >= 0;
            if (!present || g >= x) break;
            if (nc == DUPLEX_CHAIN) { atomicOr(seq, 1u); break; }
            ++nc;
            x = g;
        }
        int32_t dx = present ? 0 : 1;
        for (int k = nc - 1; k >= 0; --k) {
            if (dx == 0) dx = 2;
            else if (dx == 1) { atomicOr(err, EB_KEYERROR); dx = 3; }
            else dx = 0;
        }
        d = dx;
        if (d == 0) pr = p[i];
    } else {
        if (p[i] >= 0 && indeg[p[i]] > 1) atomicOr(seq, 1u);
        int32_t x = (int32_t)i;
        int nc = 0, dx = 3;
        bool comp = false;
        while (true) {
            const int32_t s = xs[x] >= 0 && xfirst[xs[x]] == x ? xs[x] : -1;
            const int32_t g = p[x];
            if (s >= 0) { dx = 1; break; }
            if (g < 0) { dx = 3; break; }
            if (g == x) { atomicOr(seq, 1u); break; }   // its own complement: the serial pass raises
            if (g > x) { dx = 2; comp = false; break; }
            if (nc == DUPLEX_CHAIN) { atomicOr(seq, 1u); break; }
            ++nc;
            x = g;
        }
        for (int k = nc - 1; k >= 0; --k) {
            const bool deleted = dx == 1 || dx == 3 || (dx == 2 && comp);
            if (deleted) { dx = 3; comp = false; }
            else { comp = dx == 2 && !comp; dx = 2; }
        }
        d = dx == 1 ? 0 : dx == 2 ? 1 : 2;
        pr = d == 0 ? xs[i] : d == 1 ? p[i] : -1;
    }
    dec[i] = d;
    part[i] = pr;
}

// The same decisions by one thread in processing order, the reference's dictionaries as flags
// (DCS_maker.py:245-282: duplex_dict = used, read_dict deletions = gone; singleton_correction.py:
// 278-319: sscs_dict / singleton_dict deletions, correction_dict): any fan-in, any chain length.
__global__ __launch_bounds__(64) void k_join_serial(int64_t n, int64_t m, int mode, const int32_t* __restrict__ p,
                                                    const int32_t* __restrict__ xs, uint8_t* __restrict__ used,
                                                    uint8_t* __restrict__ gone, uint8_t* __restrict__ xgone,
                                                    int32_t* __restrict__ dec, int32_t* __restrict__ part,
                                                    uint32_t* __restrict__ err) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    for (int64_t i = 0; i < n; ++i) { used[i] = 0; gone[i] = 0; }
    for (int64_t k = 0; k < m; ++k) xgone[k] = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int32_t j = p[i];
        int32_t d, pr = -1;
        if (mode == 0) {
            if (j >= 0 && used[j]) {
                d = 2;                                     // ds in duplex_dict: skipped, read_dict kept
            } else {
                if (j >= 0) {
                    if (gone[j]) { atomicOr(err, EB_KEYERROR); dec[i] = 3; part[i] = -1; return; }
                    d = 0; pr = j; used[i] = 1;
                } else {
                    d = 1;
                }
                gone[i] = 1;                               // del read_dict[tag]
            }
        } else {
            const int32_t s = xs[i];
            if (s >= 0 && !xgone[s]) {
                d = 0; pr = s; xgone[s] = 1; gone[i] = 1;
            } else if (j >= 0 && !gone[j]) {
                d = 1; pr = j;
                used[i] = 1;                               // correction_dict[tag] = duplex
                if (used[j]) {
                    if (j == (int32_t)i) { atomicOr(err, EB_KEYERROR); dec[i] = 3; part[i] = -1; return; }
                    gone[i] = gone[j] = 1;
                    used[i] = used[j] = 0;
                }
            } else {
                d = 2;
                gone[i] = 1;
            }
        }
        dec[i] = d;
        part[i] = pr;
    }
}

int upload_keys(cc_ctx* ctx, Group& g, const char* name, const void* keys, int64_t n, int kw, uint32_t** out) {
    int brc = 0;
    uint32_t* d = GB(uint32_t, name, n * kw);
    if (n > 0) HIPCHK(hipMemcpyAsync(d, keys, sizeof(uint32_t) * kw * n, hipMemcpyHostToDevice, ctx->stream));
    *out = d;
    return 0;
}

// an empty table of at least twice n slots; returns its mask
int key_table(cc_ctx* ctx, Group& g, const char* name, int64_t n, int32_t** out, uint64_t* mask) {
    int brc = 0;
    uint64_t size = 1024;
    while (size < (uint64_t)(2 * n)) size <<= 1;
    int32_t* t = GB(int32_t, name, (int64_t)size);
    HIPCHK(hipMemsetAsync(t, 0xff, sizeof(int32_t) * size, ctx->stream));
    *out = t;
    *mask = size - 1;
    return 0;
}

bool key_args_ok(cc_ctx* ctx, int32_t key_bytes) {
    if (key_bytes <= 0 || (key_bytes & 3) || key_bytes > 4 * KEY_MAX_WORDS) {
        ctx->err = "key_bytes must be a positive multiple of 4, at most 256";
        return false;
    }
    return true;
}
}  // namespace

extern "C" {

// read_dict's grouping (consensus_helper.py:426-500: read_dict[tag].append in pair-completion order,
// tag_dict insertion order) on caller-given keys: families in order of their first key, members in
// input order.
int cc_group(cc_ctx* ctx, int64_t n, const void* keys, int32_t key_bytes, int32_t* out_perm, int64_t* out_fam_offsets,
             int64_t* out_nfam) {
    if (!ctx || n < 0 || n >= INT32_MAX || !out_nfam || (n > 0 && (!keys || !out_perm || !out_fam_offsets)))
        return CC_E_INVALID;
    if (!key_args_ok(ctx, key_bytes)) return CC_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    *out_nfam = 0;
    if (n == 0) {
        if (out_fam_offsets) out_fam_offsets[0] = 0;
        return 0;
    }
    const int kw = key_bytes / 4;
    Group& g = scratch_group(ctx, -1);
    int brc = 0;
    uint32_t* dk = nullptr;
    RC(upload_keys(ctx, g, "grp_keys", keys, n, kw, &dk));
    int32_t* tab = nullptr;
    uint64_t mask = 0;
    RC(key_table(ctx, g, "grp_tab", n, &tab, &mask));
    int32_t* slot_of = GB(int32_t, "grp_slot_of", n);
    int32_t* slot_first = GB(int32_t, "grp_slot_first", (int64_t)mask + 1);
    int32_t* slot_cnt = GB(int32_t, "grp_slot_cnt", (int64_t)mask + 1);
    uint32_t* start = GB(uint32_t, "grp_start", (n + 3) & ~3LL);
    uint32_t* fx = GB(uint32_t, "grp_fx", (n + 3) & ~3LL);
    uint32_t* fam_size = GB(uint32_t, "grp_fsize", (n + 3) & ~3LL);
    uint32_t* fam_off = GB(uint32_t, "grp_foff", (n + 3) & ~3LL);
    uint64_t* fkey = GB(uint64_t, "grp_fkey", n);
    uint32_t* fval = GB(uint32_t, "grp_fval", n);
    uint64_t* skey = GB(uint64_t, "grp_skey", n);
    uint32_t* sval = GB(uint32_t, "grp_sval", n);
    {
        Fills fill(ctx);
        RC(fill.add(slot_first, sizeof(int32_t) * (mask + 1), 0x7fffffffu));
        RC(fill.add(slot_cnt, sizeof(int32_t) * (mask + 1), 0u));
        RC(fill.add(start, sizeof(uint32_t) * ((n + 3) & ~3LL), 0u));
        RC(fill.add(fam_size, sizeof(uint32_t) * ((n + 3) & ~3LL), 0u));
        RC(fill.launch());
    }
    hipLaunchKernelGGL(k_key_insert, dim3(nblk(n)), dim3(256), 0, ctx->stream, n, (const uint32_t*)dk, kw,
                       (uint64_t)0x243f6a8885a308d3ULL, tab, mask, slot_of, slot_first, slot_cnt, (uint32_t*)nullptr);
    hipLaunchKernelGGL(k_group_starts, dim3(nblk(n)), dim3(256), 0, ctx->stream, n, (const int32_t*)slot_of,
                       (const int32_t*)slot_first, start);
    int64_t F = 0;
    RC(scan_total(ctx, g, start, fx, n, &F, "grp_scan_fam"));
    hipLaunchKernelGGL(k_group_fams, dim3(nblk(n)), dim3(256), 0, ctx->stream, n, (const int32_t*)slot_of,
                       (const int32_t*)slot_first, (const int32_t*)slot_cnt, (const uint32_t*)fx, fam_size, fkey, fval);
    int64_t tot = 0;
    RC(scan_total(ctx, g, fam_size, fam_off, F, &tot, "grp_scan_off"));
    // members in input order inside their family: a stable sort by family number (radix sorts are
    // stable; the values enter in input order)
    unsigned bits = 1;
    while (bits < 32 && (1ULL << bits) < (uint64_t)F) ++bits;
    RC(sort_pairs(ctx, fkey, skey, fval, sval, n, "sort_group", 0u, bits));
    std::vector<uint32_t> off((size_t)F);
    HIPCHK(hipMemcpyAsync(out_perm, sval, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(off.data(), fam_off, sizeof(uint32_t) * F, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (int64_t f = 0; f < F; ++f) out_fam_offsets[f] = off[f];
    out_fam_offsets[F] = n;
    *out_nfam = F;
    return tot == n ? 0 : CC_E_INVALID;
}

// The duplex pairing of DCS_maker.py:245-282 (mode 0) and singleton_correction.py:278-319 (mode 1)
// on caller-given tags (see the header).
int cc_duplex_join(cc_ctx* ctx, int32_t mode, int64_t n, const void* keys, const void* partner_keys, int64_t m,
                   const void* x_keys, int32_t key_bytes, int32_t* out_decision, int64_t* out_partner, int32_t table_a,
                   const int32_t* rec_a, int32_t table_x, const int32_t* rec_x, uint8_t* out_seq, uint8_t* out_qual,
                   int32_t* out_meta, int32_t out_stride) {
    if (!ctx || (mode != 0 && mode != 1) || n < 0 || n >= INT32_MAX || m < 0 || m >= INT32_MAX ||
        (n > 0 && (!keys || !partner_keys || !out_decision || !out_partner)) || (mode == 1 && m > 0 && !x_keys))
        return CC_E_INVALID;
    if (!key_args_ok(ctx, key_bytes)) return CC_E_INVALID;
    const bool vote = out_seq != nullptr;
    if (vote) {
        if (!out_qual || !out_meta || !rec_a || !ctx->tables.count(table_a) ||
            (mode == 1 && m > 0 && (!rec_x || !ctx->tables.count(table_x)))) return CC_E_INVALID;
        const int32_t ml = std::max(ctx->tables[table_a].max_len, mode == 1 && m > 0 ? ctx->tables[table_x].max_len : 0);
        if (out_stride < ml || (out_stride & 1)) {
            ctx->err = "out_stride must be even and at least the tables' longest read";
            return CC_E_INVALID;
        }
        for (int64_t i = 0; i < n; ++i)
            if (rec_a[i] < 0 || rec_a[i] >= ctx->tables[table_a].n) { ctx->err = "rec_a outside table_a"; return CC_E_INVALID; }
        for (int64_t k = 0; mode == 1 && k < m; ++k)
            if (rec_x[k] < 0 || rec_x[k] >= ctx->tables[table_x].n) { ctx->err = "rec_x outside table_x"; return CC_E_INVALID; }
    }
    HIPCHK(hipSetDevice(ctx->device));
    if (n == 0) return 0;
    const int kw = key_bytes / 4;
    const int64_t mx = mode == 1 ? m : 0;
    Group& g = scratch_group(ctx, table_a);
    int brc = 0;
    uint32_t *dk = nullptr, *dp = nullptr, *dx = nullptr;
    RC(upload_keys(ctx, g, "join_keys", keys, n, kw, &dk));
    RC(upload_keys(ctx, g, "join_pkeys", partner_keys, n, kw, &dp));
    if (mx > 0) RC(upload_keys(ctx, g, "join_xkeys", x_keys, mx, kw, &dx));
    int32_t *tab = nullptr, *xtab = nullptr;
    uint64_t mask = 0, xmask = 0;
    RC(key_table(ctx, g, "join_tab", n, &tab, &mask));
    if (mx > 0) RC(key_table(ctx, g, "join_xtab", mx, &xtab, &xmask));
    int32_t* p = GB(int32_t, "join_p", n);
    int32_t* xs = GB(int32_t, "join_xs", n);
    int32_t* xfirst = GB(int32_t, "join_xfirst", std::max<int64_t>(mx, 1));
    int32_t* indeg = GB(int32_t, "join_indeg", n);
    int32_t* dec = GB(int32_t, "join_dec", n);
    int32_t* part = GB(int32_t, "join_part", n);
    uint32_t* flags = GB(uint32_t, "join_flags", 4);   // [0] duplicate key, [1] serial needed
    uint8_t* used = GB(uint8_t, "join_used", n);
    uint8_t* gone = GB(uint8_t, "join_gone", n);
    uint8_t* xgone = GB(uint8_t, "join_xgone", std::max<int64_t>(mx, 1));
    {
        Fills fill(ctx);
        RC(fill.add(xs, sizeof(int32_t) * n, ~0u));
        RC(fill.add(xfirst, sizeof(int32_t) * std::max<int64_t>(mx, 1), 0x7fffffffu));
        RC(fill.add(indeg, sizeof(int32_t) * n, 0u));
        RC(fill.add(flags, 16, 0u));
        RC(fill.add(ctx->d_err, 64, 0u));
        RC(fill.launch());
    }
    const uint64_t seed = 0x13198a2e03707344ULL;
    hipLaunchKernelGGL(k_key_insert, dim3(nblk(n)), dim3(256), 0, ctx->stream, n, (const uint32_t*)dk, kw, seed, tab, mask,
                       (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr, flags);
    hipLaunchKernelGGL(k_key_probe, dim3(nblk(n)), dim3(256), 0, ctx->stream, n, (const uint32_t*)dp, (const uint32_t*)dk,
                       kw, seed, (const int32_t*)tab, mask, p, (int32_t*)nullptr, indeg);
    if (mx > 0) {
        hipLaunchKernelGGL(k_key_insert, dim3(nblk(mx)), dim3(256), 0, ctx->stream, mx, (const uint32_t*)dx, kw, seed, xtab,
                           xmask, (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr, flags);
        hipLaunchKernelGGL(k_key_probe, dim3(nblk(n)), dim3(256), 0, ctx->stream, n, (const uint32_t*)dp,
                           (const uint32_t*)dx, kw, seed, (const int32_t*)xtab, xmask, xs, xfirst, (int32_t*)nullptr);
    }
    hipLaunchKernelGGL(k_join_decide, dim3(nblk(n)), dim3(256), 0, ctx->stream, n, mode, (const int32_t*)p,
                       (const int32_t*)xs, (const int32_t*)xfirst, (const int32_t*)indeg, dec, part, flags + 1, ctx->d_err);
    uint32_t hf[4] = {0, 0, 0, 0};
    HIPCHK(hipMemcpyAsync(hf, flags, 16, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (hf[0]) { ctx->err = "duplicate key (the tags of one call must be distinct)"; return CC_E_INVALID; }
    if (hf[1]) {
        Fills fill(ctx);
        RC(fill.add(ctx->d_err, 64, 0u));
        RC(fill.launch());
        hipLaunchKernelGGL(k_join_serial, dim3(1), dim3(64), 0, ctx->stream, n, mx, mode, (const int32_t*)p,
                           (const int32_t*)xs, used, gone, xgone, dec, part, ctx->d_err);
    }
    uint32_t bits = 0;
    RC(read_err(ctx, &bits));
    if (bits) return err_code(ctx, bits);
    std::vector<int32_t> hd((size_t)n), hp((size_t)n);
    HIPCHK(hipMemcpyAsync(hd.data(), dec, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(hp.data(), part, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (int64_t i = 0; i < n; ++i) {
        out_decision[i] = hd[i];
        out_partner[i] = hp[i];
    }
    if (!vote) return 0;
    // the consensus of every joined pair (DCS: decision 0; SC: 0 and 1), row i for entry i
    std::vector<int32_t> ta, pb, dv, rows;
    for (int64_t i = 0; i < n; ++i) {
        const bool v = mode == 0 ? hd[i] == 0 : hd[i] <= 1;
        if (!v) continue;
        ta.push_back(rec_a[i]);
        pb.push_back(mode == 1 && hd[i] == 0 ? rec_x[hp[i]] : rec_a[hp[i]]);
        dv.push_back(mode == 1 ? hd[i] : 1);   // k_duplex_vote_swar: SC decision 1 reads read2 from table A
        rows.push_back((int32_t)i);
    }
    const int64_t nv = (int64_t)ta.size();
    if (nv == 0) return 0;
    const DevTable TA = ctx->tables[table_a];
    const DevTable TX = (mode == 1 && m > 0) ? ctx->tables[table_x] : TA;
    const int32_t ml = std::max(TA.max_len, TX.max_len);
    const int32_t qstride = (int32_t)((ml + 15) & ~15);
    int4* vpair = GB(int4, "vpair", nv);
    uint8_t* cons_seq = GB(uint8_t, "cons_seq", nv * (qstride / 2));
    uint8_t* cons_qual = GB(uint8_t, "cons_qual", nv * qstride);
    int32_t* vmeta = GB(int32_t, "vote_meta", 5 * nv);
    std::vector<int4> vp((size_t)nv);
    for (int64_t k = 0; k < nv; ++k) vp[k] = make_int4(ta[k], pb[k], dv[k], (int32_t)k);
    HIPCHK(hipMemcpyAsync(vpair, vp.data(), sizeof(int4) * nv, hipMemcpyHostToDevice, ctx->stream));
    {
        Fills fill(ctx);
        RC(fill.add(ctx->d_err, 64, 0u));
        RC(fill.launch());
    }
    RC(function_prep(ctx, TA));
    if (TX.payload != TA.payload) RC(function_prep(ctx, TX));
    {
        ProfScope ps(ctx, mode ? "k_duplex_vote_sc" : "k_duplex_vote_dcs");
        const int32_t chunks = std::min(64, std::max(1, (ml + SV_POS - 1) / SV_POS));
        const int32_t fpw = 64 / chunks;
        hipLaunchKernelGGL(k_duplex_vote_swar, dim3(nblk((nv + fpw - 1) / fpw, 4)), dim3(256), 0, ctx->stream, nv, mode,
                           fpw, chunks, (const int4*)vpair, TA, TX, qstride, cons_seq, cons_qual, vmeta, ctx->d_err);
    }
    RC(read_err(ctx, &bits));
    if (bits) return err_code(ctx, bits);
    std::vector<uint8_t> hq((size_t)nv * qstride), hs((size_t)nv * (qstride / 2));
    std::vector<int32_t> hm((size_t)nv * 5);
    HIPCHK(hipMemcpyAsync(hq.data(), cons_qual, hq.size(), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(hs.data(), cons_seq, hs.size(), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(hm.data(), vmeta, sizeof(int32_t) * hm.size(), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    for (int64_t k = 0; k < nv; ++k) {
        const int64_t i = rows[k];
        memcpy(out_qual + i * (int64_t)out_stride, hq.data() + k * qstride, (size_t)ml);
        memcpy(out_seq + i * (int64_t)(out_stride / 2), hs.data() + k * (qstride / 2), (size_t)((ml + 1) / 2));
        memcpy(out_meta + 5 * i, hm.data() + 5 * k, sizeof(int32_t) * 5);
    }
    return 0;
}

}  // extern "C"

// ------------------------------------------------------------------ fastq2bam UMI extraction (f4)
// extract_barcodes.py:287-405's per-pair decision on the GPU (libccio's ccio_fq_* read the FASTQs and
// write the outputs).  One thread per read pair over the first EB_W bases of both reads:
//   pattern mode (:294-337): a non-ACGT base in either read's first len(pattern) bases -> bad barcode
//     (2); the per-position base histogram; a spacer base differing in either read -> missing spacer
//     (1); else passing (0), barcode = the N positions of read 1 '.' those of read 2, both reads cut by
//     len(pattern);
//   list mode (:339-405): for each distinct barcode length, longest first, the reads' prefixes
//     (read.seq[:blen]): a non-ACGT prefix counts a bad barcode and goes to the read's bad list
//     (mask bit j), else a listed prefix is that read's match (a later, shorter match replaces it);
//     both reads matched -> passing, barcode = match minus its final T per read, reads cut by their
//     matches' lengths, the list entries counted; else a bad barcode, and the unmatched reads'
//     shortest-length prefixes go to the bad lists (mask bit 31).
constexpr int EB_W = 32;           // bases of each read the decision reads (barcode lengths <= 32)
constexpr int EB_BC = 2 * EB_W + 8;  // barcode string bytes per pair (NUL terminated)
constexpr int EB_MAXLIST = 1024, EB_SLOTS = 2 * EB_MAXLIST;   // 32 KB of LDS
struct EbParams {
    int32_t list;              // 0 pattern, 1 list
    int32_t plen, nb, ns;      // pattern: length, N positions, spacer positions
    int8_t bidx[EB_W], sidx[EB_W];
    char spacer[EB_W];
    int32_t nlens, lens[EB_W]; // list: the distinct lengths, longest first
    int32_t nlist;
};
__device__ __forceinline__ int eb_code(uint8_t c) {
    return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : 4;
}
__device__ __forceinline__ uint64_t eb_slot_hash(uint64_t packed, int k) { return mix64(packed * 64 + (uint64_t)k); }

// list entries (ACGT only, <= EB_W bases) packed 2 bits per base: the table the kernel copies to LDS
__global__ __launch_bounds__(256) void k_eb_list(int32_t nlist, const uint8_t* __restrict__ ent, const int32_t* __restrict__ elen,
                                                 unsigned long long* __restrict__ tkey, int32_t* __restrict__ tval) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlist) return;
    const int k = elen[i];
    uint64_t pk = 0;
    bool ok = k > 0 && k <= EB_W;
    for (int j = 0; j < k && ok; ++j) {
        const int c = eb_code(ent[i * EB_W + j]);
        if (c > 3) ok = false;
        pk = (pk << 2) | (uint64_t)c;
    }
    if (!ok) return;   // an entry with an N never matches a prefix that passed the ACGT check
    const unsigned long long key = (pk << 6) | (unsigned long long)k;
    uint32_t h = (uint32_t)eb_slot_hash(pk, k) & (EB_SLOTS - 1);
    for (int p = 0; p < EB_SLOTS; ++p) {
        const unsigned long long prev = atomicCAS(&tkey[h], ~0ULL, key);
        if (prev == ~0ULL) { tval[h] = i; return; }
        if (prev == key) { atomicMin(&tval[h], i); return; }   // (the host passes distinct entries)
        h = (h + 1) & (EB_SLOTS - 1);
    }
}

__global__ __launch_bounds__(256) void k_extract_barcodes(
    int64_t n, const uint8_t* __restrict__ h1, const uint8_t* __restrict__ h2, const int32_t* __restrict__ len1,
    const int32_t* __restrict__ len2, EbParams P, const unsigned long long* __restrict__ tkey,
    const int32_t* __restrict__ tval, uint8_t* __restrict__ status, char* __restrict__ bc, int32_t* __restrict__ cut1,
    int32_t* __restrict__ cut2, uint32_t* __restrict__ bad1, uint32_t* __restrict__ bad2,
    unsigned long long* __restrict__ counts, unsigned long long* __restrict__ hist1, unsigned long long* __restrict__ hist2) {
    __shared__ unsigned long long s_key[EB_SLOTS];
    __shared__ int32_t s_val[EB_SLOTS];
    __shared__ uint32_t s_h1[EB_MAXLIST], s_h2[EB_MAXLIST];   // pattern: 5 * plen bins; list: one per entry
    const int t = threadIdx.x;
    const int nh = P.list ? P.nlist : 5 * P.plen;
    if (P.list)
        for (int i = t; i < EB_SLOTS; i += blockDim.x) { s_key[i] = tkey[i]; s_val[i] = tval[i]; }
    for (int i = t; i < nh; i += blockDim.x) { s_h1[i] = 0; s_h2[i] = 0; }
    __syncthreads();
    int acc[3] = {0, 0, 0};   // missing spacer, bad barcode, passing
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + t;
    if (i < n) {
        uint8_t x[EB_W], y[EB_W];
#pragma unroll
        for (int w = 0; w < EB_W / 16; ++w) {
            *reinterpret_cast<uint4*>(x + 16 * w) = reinterpret_cast<const uint4*>(h1 + i * EB_W)[w];
            *reinterpret_cast<uint4*>(y + 16 * w) = reinterpret_cast<const uint4*>(h2 + i * EB_W)[w];
        }
        const int lx = len1[i], ly = len2[i];
        char* out = bc + i * EB_BC;
        uint8_t st = 2;
        int32_t c1 = 0, c2 = 0;
        uint32_t m1 = 0, m2 = 0;
        if (!P.list) {
            bool ok = true;
            for (int k = 0; k < P.plen; ++k) ok = ok && eb_code(x[k]) < 4 && eb_code(y[k]) < 4;
            if (!ok) {
                acc[1] += 1;
            } else {
                for (int k = 0; k < P.plen; ++k) {
                    atomicAdd(&s_h1[5 * k + eb_code(x[k])], 1u);
                    atomicAdd(&s_h2[5 * k + eb_code(y[k])], 1u);
                }
                bool sp = true;
                for (int k = 0; k < P.ns; ++k) sp = sp && x[P.sidx[k]] == (uint8_t)P.spacer[k] && y[P.sidx[k]] == (uint8_t)P.spacer[k];
                if (!sp) {
                    acc[0] += 1;
                    st = 1;
                } else {
                    acc[2] += 1;
                    st = 0;
                    int o = 0;
                    for (int k = 0; k < P.nb; ++k) out[o++] = (char)x[P.bidx[k]];
                    out[o++] = '.';
                    for (int k = 0; k < P.nb; ++k) out[o++] = (char)y[P.bidx[k]];
                    out[o] = 0;
                    c1 = c2 = P.plen;
                }
            }
        } else {
            int32_t l1 = -1, l2 = -1, e1 = -1, e2 = -1;
            for (int j = 0; j < P.nlens; ++j) {
                const int bl = P.lens[j];
                const int k1 = bl < lx ? bl : lx, k2 = bl < ly ? bl : ly;
                uint64_t p1 = 0, p2 = 0;
                bool ok1 = true, ok2 = true;
                for (int k = 0; k < k1; ++k) { const int c = eb_code(x[k]); ok1 = ok1 && c < 4; p1 = (p1 << 2) | (uint64_t)(c & 3); }
                for (int k = 0; k < k2; ++k) { const int c = eb_code(y[k]); ok2 = ok2 && c < 4; p2 = (p2 << 2) | (uint64_t)(c & 3); }
                if (!ok1 || !ok2) {
                    acc[1] += 1;
                    if (!ok1) m1 |= 1u << j;
                    if (!ok2) m2 |= 1u << j;
                    continue;
                }
                for (int r = 0; r < 2; ++r) {
                    const uint64_t pk = r ? p2 : p1;
                    const int kk = r ? k2 : k1;
                    const unsigned long long key = (pk << 6) | (unsigned long long)kk;
                    uint32_t h = (uint32_t)eb_slot_hash(pk, kk) & (EB_SLOTS - 1);
                    int32_t hit = -1;
                    for (int q = 0; q < EB_SLOTS && kk > 0; ++q) {
                        const unsigned long long sk = s_key[h];
                        if (sk == ~0ULL) break;
                        if (sk == key) { hit = s_val[h]; break; }
                        h = (h + 1) & (EB_SLOTS - 1);
                    }
                    if (hit >= 0) {
                        if (r) { l2 = bl; e2 = hit; } else { l1 = bl; e1 = hit; }
                    }
                }
            }
            if (l1 > 0 && l2 > 0) {
                acc[2] += 1;
                st = 0;
                atomicAdd(&s_h1[e1], 1u);
                atomicAdd(&s_h2[e2], 1u);
                int o = 0;
                for (int k = 0; k + 1 < l1; ++k) out[o++] = (char)x[k];
                out[o++] = '.';
                for (int k = 0; k + 1 < l2; ++k) out[o++] = (char)y[k];
                out[o] = 0;
                c1 = l1;
                c2 = l2;
            } else {
                acc[1] += 1;
                if (l1 <= 0) m1 |= 1u << 31;
                if (l2 <= 0) m2 |= 1u << 31;
            }
            bad1[i] = m1;
            bad2[i] = m2;
        }
        status[i] = st;
        cut1[i] = c1;
        cut2[i] = c2;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        int v = acc[c];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((t & 63) == 0 && v) atomicAdd(&counts[c], (unsigned long long)v);
    }
    __syncthreads();
    for (int k = t; k < nh; k += blockDim.x) {
        if (s_h1[k]) atomicAdd(&hist1[k], (unsigned long long)s_h1[k]);
        if (s_h2[k]) atomicAdd(&hist2[k], (unsigned long long)s_h2[k]);
    }
}

extern "C" {

int cc_extract_barcodes(cc_ctx* ctx, int64_t n, const uint8_t* h1, const uint8_t* h2, const int32_t* len1,
                        const int32_t* len2, const char* pattern, const char* const* blist, int32_t nblist,
                        uint8_t* out_status, char* out_bc, int32_t* out_cut1, int32_t* out_cut2, uint32_t* out_bad1,
                        uint32_t* out_bad2, int64_t* counts, int64_t* r1_hist, int64_t* r2_hist) {
    if (!ctx || n < 0 || !counts || !r1_hist || !r2_hist || (!pattern && (!blist || nblist <= 0)) ||
        (n > 0 && (!h1 || !h2 || !len1 || !len2 || !out_status || !out_bc || !out_cut1 || !out_cut2)) ||
        (!pattern && n > 0 && (!out_bad1 || !out_bad2)))
        return CC_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    EbParams P;
    memset(&P, 0, sizeof P);
    P.list = pattern ? 0 : 1;
    std::vector<uint8_t> ent;
    std::vector<int32_t> elen;
    if (pattern) {
        P.plen = (int32_t)strlen(pattern);
        if (P.plen > EB_W || 5 * P.plen > EB_MAXLIST) { ctx->err = "barcode pattern longer than 32"; return CC_E_UNSUPPORTED; }
        for (int k = 0; k < P.plen; ++k) {
            if (pattern[k] == 'N') P.bidx[P.nb++] = (int8_t)k;
            else { P.sidx[P.ns] = (int8_t)k; P.spacer[P.ns++] = pattern[k]; }
        }
    } else {
        if (nblist > EB_MAXLIST) { ctx->err = "more than 1024 listed barcodes"; return CC_E_UNSUPPORTED; }
        P.nlist = nblist;
        std::vector<int32_t> lens;
        ent.assign((size_t)nblist * EB_W, 0);
        elen.assign((size_t)nblist, 0);
        for (int32_t i = 0; i < nblist; ++i) {
            const int32_t k = (int32_t)strlen(blist[i]);
            if (k > EB_W) { ctx->err = "listed barcode longer than 32"; return CC_E_UNSUPPORTED; }
            memcpy(&ent[(size_t)i * EB_W], blist[i], (size_t)k);
            elen[i] = k;
            if (std::find(lens.begin(), lens.end(), k) == lens.end()) lens.push_back(k);
        }
        std::sort(lens.rbegin(), lens.rend());
        if ((int)lens.size() > 31) { ctx->err = "more than 31 barcode lengths"; return CC_E_UNSUPPORTED; }
        P.nlens = (int32_t)lens.size();
        for (size_t j = 0; j < lens.size(); ++j) P.lens[j] = lens[j];
    }
    const int nh = P.list ? P.nlist : 5 * P.plen;
    Group& g = scratch_group(ctx, -1);
    int brc = 0;
    uint8_t* d1 = GB(uint8_t, "eb_h1", n * EB_W);
    uint8_t* d2 = GB(uint8_t, "eb_h2", n * EB_W);
    int32_t* dl1 = GB(int32_t, "eb_l1", n);
    int32_t* dl2 = GB(int32_t, "eb_l2", n);
    uint8_t* dst = GB(uint8_t, "eb_status", n);
    char* dbc = GB(char, "eb_bc", n * EB_BC);
    int32_t* dc1 = GB(int32_t, "eb_cut1", n);
    int32_t* dc2 = GB(int32_t, "eb_cut2", n);
    uint32_t* db1 = GB(uint32_t, "eb_bad1", n);
    uint32_t* db2 = GB(uint32_t, "eb_bad2", n);
    unsigned long long* dcnt = GB(unsigned long long, "eb_counts", 4);
    unsigned long long* dh = GB(unsigned long long, "eb_hist", 2 * std::max(nh, 1));
    unsigned long long* tkey = GB(unsigned long long, "eb_tkey", EB_SLOTS);
    int32_t* tval = GB(int32_t, "eb_tval", EB_SLOTS);
    uint8_t* dent = GB(uint8_t, "eb_ent", std::max<int64_t>((int64_t)ent.size(), 1));
    int32_t* delen = GB(int32_t, "eb_elen", std::max<int64_t>((int64_t)elen.size(), 1));
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(d1, h1, (size_t)n * EB_W, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(d2, h2, (size_t)n * EB_W, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(dl1, len1, sizeof(int32_t) * n, hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(dl2, len2, sizeof(int32_t) * n, hipMemcpyHostToDevice, ctx->stream));
    }
    HIPCHK(hipMemsetAsync(dcnt, 0, 32, ctx->stream));
    HIPCHK(hipMemsetAsync(dh, 0, sizeof(unsigned long long) * 2 * std::max(nh, 1), ctx->stream));
    HIPCHK(hipMemsetAsync(tkey, 0xff, sizeof(unsigned long long) * EB_SLOTS, ctx->stream));
    HIPCHK(hipMemsetAsync(tval, 0x7f, sizeof(int32_t) * EB_SLOTS, ctx->stream));
    if (P.list) {
        HIPCHK(hipMemcpyAsync(dent, ent.data(), ent.size(), hipMemcpyHostToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(delen, elen.data(), sizeof(int32_t) * elen.size(), hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_eb_list, dim3(nblk(nblist)), dim3(256), 0, ctx->stream, nblist, (const uint8_t*)dent,
                           (const int32_t*)delen, tkey, tval);
    }
    if (n > 0) {
        ProfScope ps(ctx, "k_extract_barcodes");
        hipLaunchKernelGGL(k_extract_barcodes, dim3(nblk(n)), dim3(256), 0, ctx->stream, n, (const uint8_t*)d1,
                           (const uint8_t*)d2, (const int32_t*)dl1, (const int32_t*)dl2, P,
                           (const unsigned long long*)tkey, (const int32_t*)tval, dst, dbc, dc1, dc2, db1, db2, dcnt,
                           dh, dh + std::max(nh, 1));
        HIPCHK(hipMemcpyAsync(out_status, dst, (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipMemcpyAsync(out_bc, dbc, (size_t)n * EB_BC, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipMemcpyAsync(out_cut1, dc1, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipMemcpyAsync(out_cut2, dc2, sizeof(int32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
        if (P.list) {
            HIPCHK(hipMemcpyAsync(out_bad1, db1, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(hipMemcpyAsync(out_bad2, db2, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
        }
    }
    std::vector<unsigned long long> hc(4), hh(2 * std::max(nh, 1));
    HIPCHK(hipMemcpyAsync(hc.data(), dcnt, 32, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(hh.data(), dh, sizeof(unsigned long long) * hh.size(), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    RC(dbg_fault(ctx));
    counts[0] = (int64_t)hc[0];
    counts[1] = (int64_t)hc[1];
    counts[2] = (int64_t)hc[2];
    for (int k = 0; k < nh; ++k) {
        r1_hist[k] = (int64_t)hh[k];
        r2_hist[k] = (int64_t)hh[std::max(nh, 1) + k];
    }
    return 0;
}

}  // extern "C"

// ------------------------------------------------------------------ the multi-GPU reduction (RCCL)
// the one collective of the sharded pipeline.  RCCL is resolved at run
// time (dlopen), so the library loads on hosts without it; a process that already holds an RCCL
// (torch's) gets that one back from the loader.
namespace {
typedef int (*nccl_get_id_t)(void*);
struct NcclId {   // ncclUniqueId: passed BY VALUE to ncclCommInitRank
    char internal[128];
};
typedef int (*nccl_init_rank_t)(void**, int, NcclId, int);
typedef int (*nccl_allreduce_t)(const void*, void*, size_t, int, int, void*, hipStream_t);
typedef int (*nccl_simple_t)(void);
typedef int (*nccl_destroy_t)(void*);
typedef const char* (*nccl_errstr_t)(int);
constexpr int NCCL_ID_BYTES = 128;
constexpr int NCCL_INT64 = 4, NCCL_SUM = 0, NCCL_MAX = 2, NCCL_MIN = 3;   // ncclDataType_t / ncclRedOp_t values
struct Rccl {
    void* h = nullptr;
    nccl_get_id_t get_id = nullptr;
    nccl_init_rank_t init_rank = nullptr;
    nccl_allreduce_t allreduce = nullptr;
    nccl_simple_t group_start = nullptr, group_end = nullptr;
    nccl_destroy_t destroy = nullptr;
    nccl_errstr_t errstr = nullptr;
};
Rccl* rccl(std::string* err) {
    static Rccl r;
    static bool tried = false;
    if (!tried) {
        tried = true;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (r.h) break;
        }
        if (r.h) {
            r.get_id = (nccl_get_id_t)dlsym(r.h, "ncclGetUniqueId");
            r.init_rank = (nccl_init_rank_t)dlsym(r.h, "ncclCommInitRank");
            r.allreduce = (nccl_allreduce_t)dlsym(r.h, "ncclAllReduce");
            r.group_start = (nccl_simple_t)dlsym(r.h, "ncclGroupStart");
            r.group_end = (nccl_simple_t)dlsym(r.h, "ncclGroupEnd");
            r.destroy = (nccl_destroy_t)dlsym(r.h, "ncclCommDestroy");
            r.errstr = (nccl_errstr_t)dlsym(r.h, "ncclGetErrorString");
        }
    }
    if (!r.h || !r.get_id || !r.init_rank || !r.allreduce || !r.group_start || !r.group_end || !r.destroy) {
        if (err) *err = "RCCL (librccl.so.1) not available";
        return nullptr;
    }
    return &r;
}
}  // namespace

struct cc_comm {
    void* comm = nullptr;
    int32_t world = 1, rank = 0;
};

extern "C" {

int cc_comm_unique_id(char* id, int32_t cap) {
    Rccl* r = rccl(nullptr);
    if (!r || !id || cap < NCCL_ID_BYTES) return CC_E_INVALID;
    return r->get_id(id) == 0 ? 0 : CC_E_UNSUPPORTED;
}

int cc_comm_init(cc_ctx* ctx, int32_t world, int32_t rank, const char* id, cc_comm** out) {
    if (!ctx || !out || !id || world < 1 || rank < 0 || rank >= world) return CC_E_INVALID;
    Rccl* r = rccl(&ctx->err);
    if (!r) return CC_E_UNSUPPORTED;
    HIPCHK(hipSetDevice(ctx->device));
    std::unique_ptr<cc_comm> c(new cc_comm());
    c->world = world;
    c->rank = rank;
    NcclId uid;
    memcpy(uid.internal, id, sizeof(uid.internal));
    const int rc = r->init_rank(&c->comm, world, uid, rank);
    if (rc != 0) {
        ctx->err = std::string("ncclCommInitRank: ") + (r->errstr ? r->errstr(rc) : "error");
        return CC_E_UNSUPPORTED;
    }
    *out = c.release();
    return 0;
}

int cc_comm_destroy(cc_comm* comm) {
    if (!comm) return CC_E_INVALID;
    Rccl* r = rccl(nullptr);
    if (r && comm->comm) r->destroy(comm->comm);
    delete comm;
    return 0;
}

// counters[n_counters] and fam_count[fam_len] summed, fam_first[fam_len] min-reduced over the ranks
// of comm, in place; comm NULL (one process) leaves them as they are.  fam_len must agree over the
// ranks (cc_allreduce_max first).
int cc_reduce_stats(cc_ctx* ctx, cc_comm* comm, int64_t* counters, int32_t n_counters, int64_t* fam_count,
                    int64_t* fam_first, int32_t fam_len) {
    if (!ctx || n_counters < 0 || fam_len < 0 || (n_counters > 0 && !counters) ||
        (fam_len > 0 && (!fam_count || !fam_first)))
        return CC_E_INVALID;
    if (!comm) return 0;
    Rccl* r = rccl(&ctx->err);
    if (!r) return CC_E_UNSUPPORTED;
    HIPCHK(hipSetDevice(ctx->device));
    const int64_t nsum = (int64_t)n_counters + fam_len, ntot = nsum + fam_len;
    if (ntot == 0) return 0;
    int brc = 0;
    if (!ctx->scratch) ctx->scratch.reset(new Group());
    Group& g = *ctx->scratch;
    int64_t* d = GB(int64_t, "reduce_buf", ntot);
    std::vector<int64_t> h((size_t)ntot);
    std::copy(counters, counters + n_counters, h.begin());
    if (fam_len) {
        std::copy(fam_count, fam_count + fam_len, h.begin() + n_counters);
        std::copy(fam_first, fam_first + fam_len, h.begin() + nsum);
    }
    HIPCHK(hipMemcpyAsync(d, h.data(), sizeof(int64_t) * ntot, hipMemcpyHostToDevice, ctx->stream));
    int rc = r->group_start();
    if (rc == 0 && nsum > 0) rc = r->allreduce(d, d, (size_t)nsum, NCCL_INT64, NCCL_SUM, comm->comm, ctx->stream);
    if (rc == 0 && fam_len > 0)
        rc = r->allreduce(d + nsum, d + nsum, (size_t)fam_len, NCCL_INT64, NCCL_MIN, comm->comm, ctx->stream);
    const int rc2 = r->group_end();
    if (rc || rc2) {
        ctx->err = std::string("ncclAllReduce: ") + (r->errstr ? r->errstr(rc ? rc : rc2) : "error");
        return CC_E_UNSUPPORTED;
    }
    HIPCHK(hipMemcpyAsync(h.data(), d, sizeof(int64_t) * ntot, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    std::copy(h.begin(), h.begin() + n_counters, counters);
    if (fam_len) {
        std::copy(h.begin() + n_counters, h.begin() + nsum, fam_count);
        std::copy(h.begin() + nsum, h.end(), fam_first);
    }
    return 0;
}

// v[n] max-reduced over the ranks of comm, in place (the family table's length, step times)
int cc_allreduce_max(cc_ctx* ctx, cc_comm* comm, int64_t* v, int32_t n) {
    if (!ctx || n < 0 || (n > 0 && !v)) return CC_E_INVALID;
    if (!comm || n == 0) return 0;
    Rccl* r = rccl(&ctx->err);
    if (!r) return CC_E_UNSUPPORTED;
    HIPCHK(hipSetDevice(ctx->device));
    int brc = 0;
    if (!ctx->scratch) ctx->scratch.reset(new Group());
    Group& g = *ctx->scratch;
    int64_t* d = GB(int64_t, "reduce_max", n);
    HIPCHK(hipMemcpyAsync(d, v, sizeof(int64_t) * n, hipMemcpyHostToDevice, ctx->stream));
    const int rc = r->allreduce(d, d, (size_t)n, NCCL_INT64, NCCL_MAX, comm->comm, ctx->stream);
    if (rc) {
        ctx->err = std::string("ncclAllReduce: ") + (r->errstr ? r->errstr(rc) : "error");
        return CC_E_UNSUPPORTED;
    }
    HIPCHK(hipMemcpyAsync(v, d, sizeof(int64_t) * n, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return 0;
}

}  // extern "C"
