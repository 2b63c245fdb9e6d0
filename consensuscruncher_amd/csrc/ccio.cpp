// ccio.cpp — host-side BAM I/O for the MI355X consensus engine.
//
// Replaces what pysam/htslib (BAM decode/encode) do for the reference's stage
// scripts (consensus_helper.py:25, SSCS_maker.py:233-244, DCS_maker.py:162-176,
// singleton_correction.py:146-164).  pysam is not in this image, and decoding
// records into struct-of-arrays is the host half of the boundary
// (SURVEY.md §8(a) a1, §7 step 6).
//
//  * BGZF inflate/deflate, block-parallel over a std::thread pool;
//  * BAM header + record codec;
//  * decode to the SoA the GPU consumes (cc_records in include/), with exact
//    string interning of barcodes / cigar strings / RG values (ids, never hashes);
//  * qname formatting for consensus records (sscs_qname, consensus_helper.py:199-249;
//    dcs_consensus_tag, DCS_maker.py:60-96);
//  * output record assembly (create_aligned_segment, consensus_helper.py:568-619)
//    and BGZF writing.
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <map>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/consensuscruncher_amd.h"

namespace {

thread_local std::string g_err;

void set_err(const std::string& s) { g_err = s; }

// CCIO_W_ASYNC outputs still being compressed and written (finish_stream): a path-taking entry point
// waits for a pending write of its path first, ccio_flush for all of them
struct PendingWrite {
    std::string path;   // absolute
    std::shared_future<int> done;
    std::shared_ptr<std::string> err;
};
std::mutex g_pend_mu;
std::vector<PendingWrite> g_pend;

std::string abs_path(const char* p) {
    if (!p) return std::string();
    if (p[0] == '/') return std::string(p);
    char cwd[4096];
    if (!getcwd(cwd, sizeof(cwd))) return std::string(p);
    return std::string(cwd) + "/" + p;
}
// waits for the pending write of path (or of the BAM whose index path is)
void wait_path(const char* path) {
    if (!path) return;
    const std::string a = abs_path(path);
    std::vector<std::shared_future<int>> w;
    {
        std::lock_guard<std::mutex> lk(g_pend_mu);
        for (const PendingWrite& p : g_pend)
            if (p.path == a || p.path + ".bai" == a) w.push_back(p.done);
    }
    for (auto& f : w) f.wait();
}

// CCIO_TIMING=1: per-phase wall times of the writers on stderr (profiling aid)
struct PhaseTimer {
    bool on = getenv("CCIO_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char* what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "[ccio] %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

int hw_threads(int want) {
    if (want > 0) return want;
    unsigned h = std::thread::hardware_concurrency();
    if (h == 0) h = 4;
    return (int)std::min<unsigned>(h, 16);
}

void parallel_for(int64_t n, int nthreads, const std::function<void(int64_t, int64_t, int)>& fn) {
    nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<int64_t>(1, n)));
    if (nthreads == 1) {
        fn(0, n, 0);
        return;
    }
    std::vector<std::thread> th;
    int64_t chunk = (n + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; ++t) {
        int64_t b = t * chunk, e = std::min<int64_t>(n, b + chunk);
        if (b >= e) break;
        th.emplace_back(fn, b, e, t);
    }
    for (auto& x : th) x.join();
}

// ------------------------------------------------------------------ BGZF
const uint8_t kBgzfEof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43,
                              2,    0,    0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

// Raw DEFLATE for the BGZF members: libdeflate when the image has it (libdeflate.so.0, loaded at
// run time: 2-3x zlib's speed for both directions and a carry-less-multiply CRC32), else zlib.  The
// BGZF framing, and so every output file's records, do not depend on which one runs.
struct Deflate {
    void* (*alloc_d)() = nullptr;
    int (*decompress)(void*, const void*, size_t, void*, size_t, size_t*) = nullptr;
    void (*free_d)(void*) = nullptr;
    void* (*alloc_c)(int) = nullptr;
    size_t (*compress)(void*, const void*, size_t, void*, size_t) = nullptr;
    void (*free_c)(void*) = nullptr;
    uint32_t (*crc)(uint32_t, const void*, size_t) = nullptr;
    bool ok = false;
    Deflate() {
        if (getenv("CCIO_ZLIB")) return;   // zlib only (tests of the fallback)
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc_d = (void* (*)())dlsym(h, "libdeflate_alloc_decompressor");
        decompress = (int (*)(void*, const void*, size_t, void*, size_t, size_t*))dlsym(h, "libdeflate_deflate_decompress");
        free_d = (void (*)(void*))dlsym(h, "libdeflate_free_decompressor");
        alloc_c = (void* (*)(int))dlsym(h, "libdeflate_alloc_compressor");
        compress = (size_t (*)(void*, const void*, size_t, void*, size_t))dlsym(h, "libdeflate_deflate_compress");
        free_c = (void (*)(void*))dlsym(h, "libdeflate_free_compressor");
        crc = (uint32_t (*)(uint32_t, const void*, size_t))dlsym(h, "libdeflate_crc32");
        ok = alloc_d && decompress && free_d && alloc_c && compress && free_c && crc;
    }
};
const Deflate& deflate_lib() {
    static Deflate d;
    return d;
}

// one thread's codec state (a libdeflate (de)compressor or a zlib stream), made on first use
struct Codec {
    const Deflate& L = deflate_lib();
    void* dec = nullptr;
    void* enc = nullptr;
    int enc_level = -1;
    z_stream zi{}, zo{};
    bool zi_ok = false, zo_ok = false;
    int zo_level = -1;
    ~Codec() {
        if (dec) L.free_d(dec);
        if (enc) L.free_c(enc);
        if (zi_ok) inflateEnd(&zi);
        if (zo_ok) deflateEnd(&zo);
    }
    // exactly out_n bytes from in
    bool inflate_raw(const uint8_t* in, size_t in_n, uint8_t* out, size_t out_n) {
        if (L.ok) {
            if (!dec) dec = L.alloc_d();
            return dec && L.decompress(dec, in, in_n, out, out_n, nullptr) == 0;
        }
        if (!zi_ok) {
            if (inflateInit2(&zi, -15) != Z_OK) return false;
            zi_ok = true;
        }
        inflateReset(&zi);
        zi.next_in = const_cast<uint8_t*>(in);
        zi.avail_in = (uInt)in_n;
        zi.next_out = out;
        zi.avail_out = (uInt)out_n;
        return inflate(&zi, Z_FINISH) == Z_STREAM_END && zi.avail_out == 0;
    }
    // compressed size, 0 on failure
    size_t deflate_raw(int level, const uint8_t* in, size_t n, uint8_t* out, size_t cap) {
        if (L.ok) {
            const int lv = std::max(0, std::min(level, 12));
            if (!enc || enc_level != lv) {
                if (enc) L.free_c(enc);
                enc = L.alloc_c(lv);
                enc_level = lv;
            }
            return enc ? L.compress(enc, in, n, out, cap) : 0;
        }
        if (!zo_ok || zo_level != level) {
            if (zo_ok) deflateEnd(&zo);
            zo_ok = deflateInit2(&zo, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) == Z_OK;
            zo_level = level;
            if (!zo_ok) return 0;
        }
        deflateReset(&zo);
        zo.next_in = const_cast<uint8_t*>(in);
        zo.avail_in = (uInt)n;
        zo.next_out = out;
        zo.avail_out = (uInt)cap;
        if (deflate(&zo, Z_FINISH) != Z_STREAM_END) return 0;
        return cap - zo.avail_out;
    }
    uint32_t crc32_of(const uint8_t* p, size_t n) const {
        return L.ok ? L.crc(0, p, n) : (uint32_t)crc32(0L, p, (uInt)n);
    }
};

// Work-shared loop: threads take chunks of `grain` items until none are left (BGZF blocks differ
// in cost; a static split leaves threads idle).
void parallel_chunks(int64_t n, int nthreads, int64_t grain, const std::function<void(int64_t, int64_t)>& fn) {
    nthreads = std::max(1, std::min<int>(nthreads, (int)std::max<int64_t>(1, (n + grain - 1) / grain)));
    std::atomic<int64_t> next(0);
    auto work = [&]() {
        for (;;) {
            const int64_t b = next.fetch_add(grain);
            if (b >= n) break;
            fn(b, std::min(n, b + grain));
        }
    };
    if (nthreads == 1) { work(); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(work);
    for (auto& x : th) x.join();
}

template <class CVec, class Vec>
bool bgzf_inflate_all(const CVec& comp, Vec& out, int nthreads, std::string& err) {
    struct Blk { size_t coff, clen, doff, dlen; };
    std::vector<Blk> blocks;
    size_t off = 0, total = 0;
    while (off + 18 <= comp.size()) {
        const uint8_t* p = comp.data() + off;
        if (p[0] != 0x1f || p[1] != 0x8b || p[2] != 8 || !(p[3] & 4)) {
            err = "not a BGZF file (bad gzip member header)";
            return false;
        }
        uint16_t xlen = p[10] | (p[11] << 8);
        size_t bsize = 0;
        size_t x = 12;
        while (x + 4 <= 12 + (size_t)xlen && off + x + 4 <= comp.size()) {
            uint8_t si1 = p[x], si2 = p[x + 1];
            uint16_t slen = p[x + 2] | (p[x + 3] << 8);
            if (si1 == 66 && si2 == 67 && slen == 2 && off + x + 6 <= comp.size())
                bsize = (size_t)(p[x + 4] | (p[x + 5] << 8)) + 1;
            x += 4 + slen;
        }
        const size_t hdr = 12 + (size_t)xlen;
        if (bsize == 0 || off + bsize > comp.size() || bsize < hdr + 8) {
            err = "BGZF block without BC field or truncated";
            return false;
        }
        const uint8_t* tail = p + bsize - 4;
        size_t isize = (size_t)tail[0] | ((size_t)tail[1] << 8) | ((size_t)tail[2] << 16) | ((size_t)tail[3] << 24);
        blocks.push_back({off + hdr, bsize - hdr - 8, total, isize});
        total += isize;
        off += bsize;
    }
    out.resize(total);   // Vec's allocator leaves bytes uninitialised: every one is inflated below
    std::atomic<bool> bad(false);
    parallel_chunks((int64_t)blocks.size(), nthreads, 16, [&](int64_t b, int64_t e) {
        Codec c;
        for (int64_t i = b; i < e && !bad; ++i) {
            const Blk& k = blocks[i];
            if (k.dlen == 0) continue;
            if (!c.inflate_raw(comp.data() + k.coff, k.clen, out.data() + k.doff, k.dlen)) bad = true;
        }
    });
    if (bad) {
        err = "BGZF inflate failed";
        return false;
    }
    return true;
}

bool bgzf_deflate_blocks(FILE* f, const uint8_t* data, size_t n, int level, int nthreads,
                         std::vector<uint64_t>* csize = nullptr);

bool bgzf_deflate_write(FILE* f, const uint8_t* data, size_t n, int level, int nthreads,
                        std::vector<uint64_t>* csize = nullptr) {
    return bgzf_deflate_blocks(f, data, n, level, nthreads, csize) && fwrite(kBgzfEof, 1, 28, f) == 28;
}

// the BGZF members of data (no EOF marker): 0xff00-byte pieces compressed in parallel into one
// staging area (a bounded slot per piece), written in order; csize gets each member's size
bool bgzf_deflate_blocks(FILE* f, const uint8_t* data, size_t n, int level, int nthreads,
                         std::vector<uint64_t>* csize) {
    const size_t step = 0xff00;
    const size_t nb = (n + step - 1) / step;
    const size_t slot = 0x10000 + 64;   // a BGZF member is at most 64 KiB
    // pieces in rounds of at most 1024 (64 MiB of staging)
    // two staging areas: a writer thread writes one round while the next is compressed
    const size_t round = 1024;
    const size_t rcap = std::min(nb, round);
    std::unique_ptr<uint8_t[]> stage2[2] = {std::unique_ptr<uint8_t[]>(new uint8_t[rcap * slot + 1]),
                                            std::unique_ptr<uint8_t[]>(new uint8_t[nb > round ? rcap * slot + 1 : 1])};
    std::vector<size_t> len2[2] = {std::vector<size_t>(rcap), std::vector<size_t>(rcap)};
    std::thread writer;
    std::atomic<bool> wbad(false);
    int cur = 0;
    for (size_t r0 = 0; r0 < nb; r0 += round, cur ^= 1) {
        const size_t r1 = std::min(nb, r0 + round);
        uint8_t* const stage = stage2[cur].get();
        std::vector<size_t>& len = len2[cur];
        std::atomic<bool> bad(false);
        parallel_chunks((int64_t)(r1 - r0), nthreads, 8, [&](int64_t b, int64_t e) {
            Codec c;
            for (int64_t j = b; j < e && !bad; ++j) {
                const size_t i = r0 + (size_t)j;
                const size_t o = i * step, ln = std::min(step, n - o);
                uint8_t* h = stage + (size_t)j * slot;
                const size_t clen = c.deflate_raw(level, data + o, ln, h + 18, slot - 26);
                if (clen == 0 || clen + 26 > 0x10000) { bad = true; break; }
                const size_t bsize = clen + 26;
                const uint8_t hd[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 66, 67, 2, 0,
                                        (uint8_t)((bsize - 1) & 0xff), (uint8_t)((bsize - 1) >> 8)};
                memcpy(h, hd, 18);
                const uint32_t crc = c.crc32_of(data + o, ln);
                uint8_t* t = h + 18 + clen;
                for (int k = 0; k < 4; ++k) t[k] = (crc >> (8 * k)) & 0xff;
                for (int k = 0; k < 4; ++k) t[4 + k] = ((uint32_t)ln >> (8 * k)) & 0xff;
                len[j] = bsize;
            }
        });
        if (writer.joinable()) writer.join();   // the previous round is written: its area is free
        if (bad || wbad) return false;
        for (size_t j = 0; j < r1 - r0; ++j)
            if (csize) csize->push_back(len[j]);
        writer = std::thread([f, stage, &len, r0, r1, slot, &wbad]() {
            for (size_t j = 0; j < r1 - r0 && !wbad; ++j)
                if (fwrite(stage + j * slot, 1, len[j], f) != len[j]) wbad = true;
        });
    }
    if (writer.joinable()) writer.join();
    return !wbad;
}

// ------------------------------------------------------------------ helpers
inline int32_t rd32(const uint8_t* p) { int32_t v; memcpy(&v, p, 4); return v; }
inline uint32_t rdu32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint16_t rdu16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }
inline void wr32(std::string& s, int32_t v) { s.append((const char*)&v, 4); }
inline void wru16(std::string& s, uint16_t v) { s.append((const char*)&v, 2); }

const char kCigOps[] = "MIDNSHP=XB";

int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

// ------------------------------------------------------------------ interner
struct Table {
    std::unordered_map<std::string, int32_t> ids;
    std::vector<std::string> strs;
    int32_t get(const std::string& s) {
        auto it = ids.find(s);
        if (it != ids.end()) return it->second;
        int32_t id = (int32_t)strs.size();
        ids.emplace(s, id);
        strs.push_back(s);
        return id;
    }
    int32_t find(const std::string& s) const {
        auto it = ids.find(s);
        return it == ids.end() ? -1 : it->second;
    }
};

}  // namespace

struct ccio_interner {
    Table t[3];                 // 0 barcode, 1 cigar string, 2 RG value
    std::vector<int32_t> bc_swap;  // duplex_tag barcode swap, by barcode id
    std::mutex mu;
};

// a byte vector whose resize leaves new bytes uninitialised (inflate targets: no serial zero fill)
template <class T>
struct NoInit : std::allocator<T> {
    template <class U> struct rebind { using other = NoInit<U>; };
    NoInit() = default;
    template <class U> NoInit(const NoInit<U>&) {}
    template <class U> void construct(U* p) { ::new ((void*)p) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
    // streams of tens of MB and more (decoded inputs, assembled outputs) on transparent huge pages:
    // the first touch faults once per 2 MiB instead of once per 4 KiB
    static constexpr size_t kHuge = (size_t)32 << 20;
    T* allocate(size_t n) {
        const size_t b = n * sizeof(T);
        if (b < kHuge) return std::allocator<T>::allocate(n);
        void* p = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        madvise(p, b, MADV_HUGEPAGE);
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t n) {
        const size_t b = n * sizeof(T);
        if (b < kHuge) std::allocator<T>::deallocate(p, n);
        else munmap(p, b);
    }
};
using Bytes = std::vector<uint8_t, NoInit<uint8_t>>;

struct ccio_bam {
    std::string header_text;
    std::vector<std::pair<std::string, int32_t>> refs;
    std::vector<uint8_t> header_raw;  // the encoded header, copied to outputs (template=)
    Bytes data;                       // decompressed stream
    std::vector<uint64_t> rec_off;    // offset of block_size of every record
    std::vector<int64_t> origin;      // ccio_bam_combine: each record's index in the combined inputs
    std::shared_future<int> pending;  // CCIO_W_ASYNC: the write of the file this handle's stream is
                                      // being compressed into (it reads `data`: waited for first)
    ~ccio_bam() {
        if (pending.valid()) pending.wait();
    }
};

namespace {

// duplex_tag's barcode swap (consensus_helper.py:663-674): around the first '.',
// else halves at len//2.
std::string swap_barcode(const std::string& b) {
    size_t d = b.find('.');
    if (d != std::string::npos) return b.substr(d + 1) + "." + b.substr(0, d);
    size_t h = b.size() / 2;
    return b.substr(h) + b.substr(0, h);
}

std::string cigar_string(const uint8_t* r) {   // r = record core (after block_size)
    uint16_t ncig = rdu16(r + 12);
    if (ncig == 0) return "None";  // pysam cigarstring -> None, formatted into tags as 'None'
    uint8_t lqn = r[8];
    const uint8_t* c = r + 32 + lqn;
    std::string s;
    char buf[16];
    for (int i = 0; i < ncig; ++i) {
        uint32_t v = rdu32(c + 4 * i);
        snprintf(buf, sizeof buf, "%u%c", v >> 4, kCigOps[(v & 0xf) < 10 ? (v & 0xf) : 0]);
        s += buf;
    }
    return s;
}

// returns value string of RG:Z / RG:A, or sets *found=0.  *bad=1 for other types.
bool find_rg(const uint8_t* aux, const uint8_t* end, std::string& val, bool& bad) {
    const uint8_t* p = aux;
    bad = false;
    while (p + 3 <= end) {
        char t0 = p[0], t1 = p[1], ty = p[2];
        p += 3;
        size_t sz = 0;
        bool is_rg = (t0 == 'R' && t1 == 'G');
        switch (ty) {
            case 'A': case 'c': case 'C': sz = 1; break;
            case 's': case 'S': sz = 2; break;
            case 'i': case 'I': case 'f': sz = 4; break;
            case 'Z': case 'H': {
                const uint8_t* q = p;
                while (q < end && *q) ++q;
                if (is_rg) {
                    if (ty != 'Z') bad = true;
                    val.assign((const char*)p, q - p);
                    return true;
                }
                p = q + 1;
                continue;
            }
            case 'B': {
                char sub = p[0];
                int32_t cnt = rd32(p + 1);
                size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
                if (is_rg) bad = true;
                p += 5 + es * (size_t)cnt;
                continue;
            }
            default: bad = true; return false;
        }
        if (is_rg) {
            if (ty == 'A') { val.assign((const char*)p, 1); return true; }
            bad = true;
            return true;
        }
        p += sz;
    }
    return false;
}

inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
// payload slot of one record: [qual | pad16][seq nibbles | pad16], the whole slot padded to
// 128 B (one HBM/L2 line) so a read of L = 150 touches two lines, not three or four
inline size_t pay_slot(int32_t lseq) { return (align16(lseq) + align16((lseq + 1) / 2) + 127) & ~(size_t)127; }

}  // namespace

extern "C" {

const char* ccio_last_error(void) { return g_err.c_str(); }

// Per value 0..maxv of v[0..n): its count and its first index (n when absent), in one pass: the
// family-size census of read_families.txt (Counter over tag_dict values in insertion order,
// SSCS_maker.py:401-408).  -1 on a value outside [0, maxv].
int ccio_value_census(const int32_t* v, int64_t n, int32_t maxv, int64_t* first, int64_t* count) {
    for (int32_t k = 0; k <= maxv; ++k) { first[k] = n; count[k] = 0; }
    for (int64_t i = 0; i < n; ++i) {
        const int32_t x = v[i];
        if (x < 0 || x > maxv) { set_err("census: value out of range"); return -1; }
        if (count[x]++ == 0) first[x] = i;
    }
    return 0;
}

// waits for every CCIO_W_ASYNC write; -1 (ccio_last_error: the first failure) when one failed
int ccio_flush(void) {
    std::vector<PendingWrite> w;
    {
        std::lock_guard<std::mutex> lk(g_pend_mu);
        w.swap(g_pend);
    }
    int rc = 0;
    for (PendingWrite& p : w)
        if (p.done.get() != 0 && rc == 0) {
            set_err(*p.err);
            rc = -1;
        }
    return rc;
}

ccio_interner* ccio_interner_new(void) { return new ccio_interner(); }
void ccio_interner_free(ccio_interner* it) { delete it; }
int64_t ccio_interner_size(ccio_interner* it, int kind) {
    if (kind < 0 || kind > 2) return -1;
    return (int64_t)it->t[kind].strs.size();
}
int ccio_interner_get(ccio_interner* it, int kind, int64_t id, char* buf, int buflen) {
    if (kind < 0 || kind > 2 || id < 0 || id >= (int64_t)it->t[kind].strs.size()) return -1;
    const std::string& s = it->t[kind].strs[id];
    int n = (int)std::min<size_t>(s.size(), (size_t)std::max(0, buflen - 1));
    memcpy(buf, s.data(), n);
    buf[n] = 0;
    return (int)s.size();
}
int32_t ccio_interner_intern(ccio_interner* it, int kind, const char* s) {
    if (kind < 0 || kind > 2) return -1;
    std::lock_guard<std::mutex> g(it->mu);
    return it->t[kind].get(s);
}
// Fills the duplex barcode-swap table (consensus_helper.py:663-674) for every
// interned barcode; swapped strings are interned too.  Returns table length.
int64_t ccio_interner_swap_table(ccio_interner* it, int32_t* out, int64_t cap) {
    Table& b = it->t[0];
    for (size_t i = 0; i < b.strs.size(); ++i) b.get(swap_barcode(b.strs[i]));
    // swapping may add strings; their swaps in turn (rotation orbits) are bounded
    for (size_t guard = 0; guard < 64; ++guard) {
        size_t before = b.strs.size();
        for (size_t i = 0; i < before; ++i) b.get(swap_barcode(b.strs[i]));
        if (b.strs.size() == before) break;
    }
    it->bc_swap.resize(b.strs.size());
    for (size_t i = 0; i < b.strs.size(); ++i) {
        int32_t s = b.find(swap_barcode(b.strs[i]));
        it->bc_swap[i] = s;  // -1 only if the orbit guard was hit
    }
    int64_t n = (int64_t)b.strs.size();
    if (out) memcpy(out, it->bc_swap.data(), sizeof(int32_t) * std::min(n, cap));
    return n;
}

}  // extern "C"

namespace {

// a plausible record at o: block_size, read name, cigar and sequence lengths consistent
inline bool record_at(const uint8_t* d, size_t n, size_t o) {
    if (o + 36 > n) return false;
    const int32_t bs = rd32(d + o);
    if (bs < 32 || o + 4 + (size_t)bs > n) return false;
    const uint8_t* r = d + o + 4;
    const uint32_t lqn = r[8];
    const uint32_t ncig = rdu16(r + 12);
    const int32_t lseq = rd32(r + 16);
    if (lqn == 0 || lseq < 0) return false;
    const uint64_t need = 32ull + lqn + 4ull * ncig + (uint64_t)(lseq + 1) / 2 + (uint64_t)lseq;
    if (need > (uint64_t)bs) return false;
    return r[32 + lqn - 1] == 0;   // the read name's NUL
}

// Record offsets of the stream d[from, n) (block_size first).  The chain of block sizes is serial by
// nature; it is walked in T pieces at once: piece t starts at the first offset past its cut where
// eight consecutive plausible records chain (record_at), and the pieces are joined where each
// chain reaches the next piece's start exactly.  A piece whose start was not a record boundary
// (the join fails) is walked again from the true boundary, so the result is always the serial
// walk's.  False for a truncated or corrupt stream.
bool scan_records(const uint8_t* d, size_t n, size_t from, int T, std::vector<uint64_t>& out) {
    out.clear();
    auto walk = [&](size_t o, size_t stop, std::vector<uint64_t>& v, size_t* end) {   // offsets < stop
        while (o < stop && o + 4 <= n) {
            __builtin_prefetch(d + o + 2048);
            const int32_t bs = rd32(d + o);
            if (bs < 32 || o + 4 + (size_t)bs > n) return false;
            v.push_back(o);
            o += 4 + (size_t)bs;
        }
        *end = o;
        return true;
    };
    const size_t span = n > from ? n - from : 0;
    const char* mn = getenv("CCIO_SCAN_MIN");   // the smallest stream walked in pieces (tests lower it)
    if (T <= 1 || span < (mn ? (size_t)atoll(mn) : ((size_t)64 << 20))) {
        size_t e = 0;
        out.reserve(span / 256 + 1024);
        return walk(from, n, out, &e);   // stops with fewer than 4 bytes left (as the serial reader did)
    }
    std::vector<size_t> start(T + 1, n);
    start[0] = from;
    parallel_chunks(T - 1, T - 1, 1, [&](int64_t a, int64_t) {
        const int t = (int)a + 1;
        size_t c = from + span * (size_t)t / (size_t)T;
        const size_t lim = std::min(n, from + span * (size_t)(t + 1) / (size_t)T);
        for (; c < lim; ++c) {
            size_t o = c;
            int k = 0;
            for (; k < 8 && record_at(d, n, o); ++k) o += 4 + (size_t)rd32(d + o);
            if (k == 8 || (k > 0 && o == n)) break;
        }
        start[t] = c < lim ? c : n;
    });
    for (int t = 1; t <= T; ++t) start[t] = std::max(start[t], start[t - 1]);
    std::vector<std::vector<uint64_t>> part(T);
    std::vector<size_t> pend(T, 0);
    std::vector<char> ok(T, 1);
    parallel_chunks(T, T, 1, [&](int64_t a, int64_t) {
        part[a].reserve((start[a + 1] - start[a]) / 256 + 16);
        ok[a] = walk(start[a], start[a + 1], part[a], &pend[a]);
    });
    out.reserve(span / 256 + 1024);
    size_t o = from;
    for (int t = 0; t < T; ++t) {
        if (o == start[t] && ok[t]) {
            out.insert(out.end(), part[t].begin(), part[t].end());
            o = pend[t];
        } else {   // the piece's start was not a boundary: walk it from the true one
            size_t e = 0;
            if (!walk(o, start[t + 1], out, &e)) return false;
            o = e;
        }
    }
    return o + 4 > n;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ reading
ccio_bam* ccio_bam_open(const char* path, int nthreads) {
    wait_path(path);
    PhaseTimer pt;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) { set_err(std::string("cannot open ") + path); return nullptr; }
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); set_err(std::string("cannot stat ") + path); return nullptr; }
    const size_t sz = (size_t)std::max<off_t>(st.st_size, 0);
    // the compressed bytes read by several threads at once (no zero fill of the buffer first)
    Bytes comp;
    comp.resize(sz);
    std::atomic<bool> short_read(false);
    parallel_chunks((int64_t)sz, hw_threads(nthreads), 64 << 20, [&](int64_t a, int64_t b) {
        size_t got = 0;
        while (got < (size_t)(b - a)) {
            const ssize_t k = pread(fd, comp.data() + a + got, (size_t)(b - a) - got, (off_t)(a + got));
            if (k <= 0) { short_read = true; return; }
            got += (size_t)k;
        }
    });
    close(fd);
    if (short_read) { set_err(std::string("short read: ") + path); return nullptr; }
    pt.lap("open: read");
    std::unique_ptr<ccio_bam> bam(new ccio_bam());
    std::string err;
    if (!bgzf_inflate_all(comp, bam->data, hw_threads(nthreads), err)) { set_err(err + ": " + path); return nullptr; }
    comp.clear();
    comp.shrink_to_fit();
    pt.lap("open: inflate");
    const Bytes& d = bam->data;
    if (d.size() < 12 || memcmp(d.data(), "BAM\1", 4) != 0) { set_err(std::string("not a BAM file: ") + path); return nullptr; }
    size_t off = 4;
    int32_t ltext = rd32(&d[off]); off += 4;
    bam->header_text.assign((const char*)&d[off], strnlen((const char*)&d[off], ltext));
    off += ltext;
    int32_t nref = rd32(&d[off]); off += 4;
    for (int i = 0; i < nref; ++i) {
        int32_t ln = rd32(&d[off]); off += 4;
        std::string name((const char*)&d[off], ln > 0 ? ln - 1 : 0);
        off += ln;
        int32_t lr = rd32(&d[off]); off += 4;
        bam->refs.emplace_back(name, lr);
    }
    bam->header_raw.assign(d.begin(), d.begin() + off);
    if (!scan_records(d.data(), d.size(), off, hw_threads(nthreads), bam->rec_off)) {
        set_err("truncated BAM record");
        return nullptr;
    }
    pt.lap("open: record walk");
    return bam.release();
}

void ccio_bam_close(ccio_bam* b) { delete b; }
int64_t ccio_bam_nrec(ccio_bam* b) { return (int64_t)b->rec_off.size(); }
int32_t ccio_bam_nref(ccio_bam* b) { return (int32_t)b->refs.size(); }
int ccio_bam_ref(ccio_bam* b, int32_t i, char* name, int cap, int32_t* len) {
    if (i < 0 || i >= (int32_t)b->refs.size()) return -1;
    snprintf(name, cap, "%s", b->refs[i].first.c_str());
    if (len) *len = b->refs[i].second;
    return 0;
}
int ccio_bam_qname(ccio_bam* b, int64_t i, char* buf, int cap) {
    if (i < 0 || i >= (int64_t)b->rec_off.size()) return -1;
    const uint8_t* r = b->data.data() + b->rec_off[i] + 4;
    return snprintf(buf, cap, "%s", (const char*)r + 32);
}

// Per-record core fields and sizes needed to size the SoA blobs.
int ccio_bam_layout(ccio_bam* b, uint64_t* qn_bytes, uint64_t* pay_bytes, int32_t* max_len, int nthreads) {
    int64_t n = (int64_t)b->rec_off.size();
    int T = hw_threads(nthreads);
    std::vector<uint64_t> qn(T, 0), pay(T, 0);
    std::vector<int32_t> ml(T, 0);
    parallel_for(n, T, [&](int64_t s, int64_t e, int t) {
        // thread-local sums (the shared arrays are written once: no false sharing in the loop)
        uint64_t q = 0, p = 0;
        int32_t m = 0;
        const uint8_t* d = b->data.data();
        const uint64_t* off = b->rec_off.data();
        for (int64_t i = s; i < e; ++i) {
            const uint8_t* r = d + off[i] + 4;
            const int32_t lseq = rd32(r + 16);
            q += (r[8] + 7) & ~7;   // l_read_name incl. NUL, 8-byte slots
            p += pay_slot(lseq);
            m = std::max(m, lseq);
        }
        qn[t] = q;
        pay[t] = p;
        ml[t] = m;
    });
    *qn_bytes = *pay_bytes = 0;
    *max_len = 0;
    for (int t = 0; t < T; ++t) { *qn_bytes += qn[t]; *pay_bytes += pay[t]; *max_len = std::max(*max_len, ml[t]); }
    return 0;
}

// 64-bit digest of a record's bytes (block_size excluded, bin zeroed): record equality for the
// "line read twice" rule (pysam compares every field of two AlignedSegments).
static uint64_t rec_digest(const uint8_t* r, int32_t bs) {
    uint64_t h = 0x9E3779B97F4A7C15ULL ^ (uint64_t)(uint32_t)bs;
    auto mix = [](uint64_t x) {
        x ^= x >> 31; x *= 0x7fb5d329728ea185ULL; x ^= x >> 27; x *= 0x81dadef4bc2dd44dULL; x ^= x >> 33;
        return x;
    };
    int32_t i = 0;
    for (; i + 8 <= bs; i += 8) {
        uint64_t w;
        memcpy(&w, r + i, 8);
        if (i == 8) w &= ~(0xffffULL << 16);   // bin
        h = mix(h ^ w) + 0x632BE59BD9B4E019ULL;
    }
    uint64_t w = 0;
    memcpy(&w, r + i, bs - i);
    if (i == 8) w &= ~(0xffffULL << 16);
    return mix(h ^ w ^ ((uint64_t)(bs - i) << 56));
}

// Decode every record into SoA.  mode 0: SSCS (barcode = qname.split(delim)[1],
// bad spacer when delim absent; consensus_helper.py:408,438-444); mode 1: duplex
// (barcode = qname.split('_')[0]; consensus_helper.py:447).
int ccio_bam_decode(ccio_bam* b, ccio_interner* it, int mode, const char* delim, cc_records* o, int nthreads) {
    int64_t n = (int64_t)b->rec_off.size();
    int T = hw_threads(nthreads);
    std::string dl = delim ? delim : "|";
    // pass 1: blob offsets (prefix sums per chunk)
    int64_t chunk = (n + T - 1) / std::max(1, T);
    std::vector<uint64_t> qbase(T + 1, 0), pbase(T + 1, 0);
    parallel_for(n, T, [&](int64_t s, int64_t e, int t) {
        uint64_t q = 0, p = 0;
        for (int64_t i = s; i < e; ++i) {
            const uint8_t* r = b->data.data() + b->rec_off[i] + 4;
            int32_t lseq = rd32(r + 16);
            q += (r[8] + 7) & ~7;
            p += pay_slot(lseq);
        }
        qbase[t + 1] = q;
        pbase[t + 1] = p;
    });
    (void)chunk;
    for (int t = 0; t < T; ++t) { qbase[t + 1] += qbase[t]; pbase[t + 1] += pbase[t]; }
    // thread-local string tables, merged afterwards (exact ids, deterministic order)
    struct Local { Table t[3]; std::vector<int32_t> ids[3]; std::string err; };
    std::vector<Local> loc(T);
    parallel_for(n, T, [&](int64_t s, int64_t e, int t) {
        Local& L = loc[t];
        for (int k = 0; k < 3; ++k) L.ids[k].resize(e - s);
        uint64_t q = qbase[t], p = pbase[t];
        std::string bc, rg, rawcig;
        // cigar ids by the raw cigar bytes (formatting the string only for a new one)
        std::unordered_map<std::string, int32_t> cig_by_raw;
        for (int64_t i = s; i < e; ++i) {
            const uint8_t* r = b->data.data() + b->rec_off[i] + 4;
            int32_t bs = rd32(r - 4);
            const uint8_t* end = r + bs;
            o->tid[i] = rd32(r + 0);
            o->pos[i] = rd32(r + 4);
            uint8_t lqn = r[8];
            o->mapq[i] = r[9];
            uint16_t ncig = rdu16(r + 12);
            o->flag[i] = rdu16(r + 14);
            int32_t lseq = rd32(r + 16);
            o->mtid[i] = rd32(r + 20);
            o->mpos[i] = rd32(r + 24);
            o->tlen[i] = rd32(r + 28);
            o->lseq[i] = lseq;
            const char* qn = (const char*)r + 32;
            size_t qlen_name = lqn > 0 ? strnlen(qn, lqn) : 0;
            // qname slot
            o->qn_off[i] = q;
            o->qn_len[i] = (uint16_t)qlen_name;
            size_t slot = (lqn + 7) & ~7;
            memset(o->qn_blob + q, 0, slot);
            memcpy(o->qn_blob + q, qn, qlen_name);
            q += slot;
            // cigar
            const uint8_t* cg = r + 32 + lqn;
            int32_t ql = -1;
            if (ncig > 0) {
                ql = 0;
                for (int c = 0; c < ncig; ++c) {
                    uint32_t v = rdu32(cg + 4 * c);
                    uint32_t op = v & 0xf;
                    if (op == 0 || op == 1 || op == 4 || op == 7 || op == 8) ql += (int32_t)(v >> 4);
                }
            }
            o->qlen[i] = ql;
            rawcig.assign((const char*)cg, 4 * (size_t)ncig);
            {
                auto ci = cig_by_raw.find(rawcig);
                if (ci == cig_by_raw.end()) ci = cig_by_raw.emplace(rawcig, L.t[1].get(cigar_string(r))).first;
                L.ids[1][i - s] = ci->second;
            }
            // payload: [qual | pad16][seq nibbles | pad16]
            const uint8_t* sq = cg + 4 * ncig;
            const uint8_t* qu = sq + (lseq + 1) / 2;
            o->pay_off[i] = p;
            size_t qa = align16(lseq);
            uint8_t* P = o->payload + p;
            memcpy(P, qu, lseq);
            memset(P + lseq, 0, qa - lseq);
            memcpy(P + qa, sq, (lseq + 1) / 2);
            memset(P + qa + (lseq + 1) / 2, 0, pay_slot(lseq) - qa - (lseq + 1) / 2);
            p += pay_slot(lseq);
            uint8_t rf = 0;
            if (lseq == 0 || qu[0] == 0xff) rf |= CC_RF_QUAL_MISSING;
            // barcode: qname.split(delim)[1] (SSCS) or qname.split('_')[0] (duplex), on the raw bytes
            auto find_from = [&](size_t from, const std::string& pat) -> size_t {
                if (pat.empty() || from > qlen_name) return std::string::npos;
                for (size_t x = from; x + pat.size() <= qlen_name; ++x) {
                    const void* hit = memchr(qn + x, pat[0], qlen_name - x - pat.size() + 1);
                    if (!hit) return std::string::npos;
                    x = (size_t)((const char*)hit - qn);
                    if (!memcmp(qn + x, pat.data(), pat.size())) return x;
                }
                return std::string::npos;
            };
            if (mode == 0) {
                const size_t d0 = find_from(0, dl);
                if (dl.empty() || d0 == std::string::npos) {
                    rf |= CC_RF_BAD_SPACER;
                    L.ids[0][i - s] = -1;
                } else {
                    const size_t st = d0 + dl.size();
                    const size_t d1 = find_from(st, dl);
                    bc.assign(qn + st, (d1 == std::string::npos ? qlen_name : d1) - st);
                    L.ids[0][i - s] = L.t[0].get(bc);
                }
            } else {
                const void* u = memchr(qn, '_', qlen_name);
                bc.assign(qn, u ? (size_t)((const char*)u - qn) : qlen_name);
                L.ids[0][i - s] = L.t[0].get(bc);
            }
            // RG
            bool bad = false;
            rg.clear();
            const uint8_t* aux = qu + lseq;
            if (find_rg(aux, end, rg, bad)) {
                if (bad) { rf |= CC_RF_RG_UNSUPPORTED; L.ids[2][i - s] = -1; }
                else L.ids[2][i - s] = L.t[2].get(rg);
            } else {
                L.ids[2][i - s] = -1;
                if (bad) rf |= CC_RF_RG_UNSUPPORTED;
            }
            o->rflags[i] = rf;
            if (o->rdig) o->rdig[i] = rec_digest(r, bs);
        }
    });
    // merge local tables into the shared interner
    std::vector<std::vector<int32_t>> remap[3];
    {
        std::lock_guard<std::mutex> g(it->mu);
        for (int k = 0; k < 3; ++k) {
            remap[k].resize(T);
            for (int t = 0; t < T; ++t) {
                auto& strs = loc[t].t[k].strs;
                remap[k][t].resize(strs.size());
                for (size_t j = 0; j < strs.size(); ++j) remap[k][t][j] = it->t[k].get(strs[j]);
            }
        }
    }
    parallel_for(n, T, [&](int64_t s, int64_t e, int t) {
        for (int64_t i = s; i < e; ++i) {
            int32_t v0 = loc[t].ids[0][i - s];
            o->bc_id[i] = v0 < 0 ? -1 : remap[0][t][v0];
            o->cigar_id[i] = remap[1][t][loc[t].ids[1][i - s]];
            int32_t v2 = loc[t].ids[2][i - s];
            o->rg_id[i] = v2 < 0 ? -1 : remap[2][t][v2];
        }
    });
    o->n = n;
    return 0;
}

// ------------------------------------------------------------------ qname formatting
// sscs_qname (consensus_helper.py:199-249) + ':' + suffix, from packed fields.
// strand: 0 pos, 1 neg, 2 None.
int64_t ccio_format_csn_names(ccio_interner* it, int64_t n, const int32_t* f9, const int64_t* suffix,
                              char* blob, int64_t cap, int64_t* off) {
    // sizes (blob NULL) and the names themselves are computed in parallel: each name's length
    // first, their offsets by a scan, then every name written at its offset
    static const char* kStrand[3] = {"pos", "neg", "None"};
    const Table& bc = it->t[0];
    const Table& cg = it->t[1];
    for (int64_t i = 0; i < n; ++i) {   // ids out of range: the reference's KeyError has no analogue
        const int32_t* f = f9 + 9 * i;
        if (f[0] < 0 || f[0] >= (int32_t)bc.strs.size() || f[5] < 0 || f[5] >= (int32_t)cg.strs.size() || f[6] < 0 ||
            f[6] >= (int32_t)cg.strs.size()) {
            set_err("name field id out of range");
            return -1;
        }
    }
    auto digits = [](int64_t v) {
        int d = v < 0 ? 2 : 1;
        uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
        while (u >= 10) { u /= 10; ++d; }
        return d;
    };
    auto put = [](char* o, int64_t v) {   // decimal of v at o; returns the end
        char tmp[24];
        int k = 0;
        uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
        do { tmp[k++] = (char)('0' + u % 10); u /= 10; } while (u);
        if (v < 0) *o++ = '-';
        while (k) *o++ = tmp[--k];
        return o;
    };
    auto length = [&](int64_t i) -> int64_t {
        const int32_t* f = f9 + 9 * i;
        int64_t l = (int64_t)bc.strs[f[0]].size();
        for (int k = 1; k <= 4; ++k) l += 1 + digits(f[k]);
        l += 1 + (int64_t)cg.strs[f[5]].size() + 1 + (int64_t)cg.strs[f[6]].size();
        l += 1 + (int64_t)strlen(kStrand[std::min(f[7] & 3, 2)]);
        l += 1 + digits((int64_t)(uint32_t)f[8]);
        l += 1 + digits(suffix[i]);
        return l;
    };
    const int T = hw_threads(0);
    parallel_chunks(n, T, 16384, [&](int64_t b0, int64_t e0) {
        for (int64_t i = b0; i < e0; ++i) off[i] = length(i);
    });
    int64_t used = 0;
    for (int64_t i = 0; i < n; ++i) { const int64_t l = off[i]; off[i] = used; used += l; }
    off[n] = used;
    if (!blob) return used;
    if (used > cap) { set_err("name blob too small"); return -1; }
    parallel_chunks(n, T, 16384, [&](int64_t b0, int64_t e0) {
        for (int64_t i = b0; i < e0; ++i) {
            const int32_t* f = f9 + 9 * i;
            char* o = blob + off[i];
            const std::string& b = bc.strs[f[0]];
            memcpy(o, b.data(), b.size()); o += b.size();
            for (int k = 1; k <= 4; ++k) { *o++ = '_'; o = put(o, f[k]); }
            const std::string& c5 = cg.strs[f[5]];
            *o++ = '_'; memcpy(o, c5.data(), c5.size()); o += c5.size();
            const std::string& c6 = cg.strs[f[6]];
            *o++ = '_'; memcpy(o, c6.data(), c6.size()); o += c6.size();
            const char* st = kStrand[std::min(f[7] & 3, 2)];
            *o++ = '_'; memcpy(o, st, strlen(st)); o += strlen(st);
            *o++ = '_'; o = put(o, (int64_t)(uint32_t)f[8]);
            *o++ = ':'; o = put(o, suffix[i]);
        }
    });
    return used;
}

// dcs_consensus_tag(tag_qname, ds_qname) (DCS_maker.py:60-96).
static std::vector<std::string> py_split(const std::string& s, char c) {
    std::vector<std::string> v;
    size_t st = 0;
    while (true) {
        size_t p = s.find(c, st);
        if (p == std::string::npos) { v.push_back(s.substr(st)); break; }
        v.push_back(s.substr(st, p - st));
        st = p + 1;
    }
    return v;
}

}  // extern "C"
namespace {
// dcs_consensus_tag (DCS_maker.py / consensus_helper.py) on the two SSCS qnames t and d, without
// allocations: barcode = t.split('_')[0], coor = t after its first '_' up to its last '_', the
// second ':' fields of both; "pos" in t orders them.  Writes the name to out (when non-null) and
// returns its length; -1 on the reference's IndexError.
int64_t dcs_name_into(const char* t, size_t tl, const char* d, size_t dl, char* out) {
    auto find = [](const char* s, size_t n, char c) -> size_t {
        const void* p = memchr(s, c, n);
        return p ? (size_t)((const char*)p - s) : n;
    };
    const size_t tb = find(t, tl, '_'), db = find(d, dl, '_');
    if (tb == tl) return -1;
    const char* rest = t + tb + 1;
    const size_t rl = tl - tb - 1;
    size_t cl = rl;   // coor = rest up to its last '_'
    for (size_t i = rl; i > 0; --i)
        if (rest[i - 1] == '_') { cl = i - 1; break; }
    const size_t t1 = find(t, tl, ':'), d1 = find(d, dl, ':');
    if (t1 == tl || d1 == dl) return -1;
    const char* tf = t + t1 + 1;
    const size_t tfl = find(tf, tl - t1 - 1, ':');
    const char* df = d + d1 + 1;
    const size_t dfl = find(df, dl - d1 - 1, ':');
    bool pos = false;
    for (size_t i = 0; i + 3 <= tl && !pos; ++i) pos = t[i] == 'p' && t[i + 1] == 'o' && t[i + 2] == 's';
    const int64_t len = (int64_t)(tb + 1 + db + 1 + cl + 1 + tfl + 1 + dfl);
    if (out) {
        char* o = out;
        auto put = [&](const char* p, size_t n) { memcpy(o, p, n); o += n; };
        if (pos) { put(t, tb); *o++ = '_'; put(d, db); }
        else { put(d, db); *o++ = '_'; put(t, tb); }
        *o++ = '_';
        put(rest, cl);
        *o++ = ':';
        if (pos) { put(tf, tfl); *o++ = '_'; put(df, dfl); }
        else { put(df, dfl); *o++ = '_'; put(tf, tfl); }
    }
    return len;
}
}  // namespace
extern "C" {

int ccio_dcs_name(const char* tag, const char* ds, char* out, int cap) {
    const int64_t k = dcs_name_into(tag, strlen(tag), ds, strlen(ds), nullptr);
    if (k < 0) { set_err("IndexError in dcs_consensus_tag"); return -1; }
    if (out && cap > 0) {
        if (k < cap) {
            dcs_name_into(tag, strlen(tag), ds, strlen(ds), out);
            out[k] = 0;
        } else {   // (snprintf's truncation)
            std::string tmp((size_t)k, '\0');
            dcs_name_into(tag, strlen(tag), ds, strlen(ds), &tmp[0]);
            memcpy(out, tmp.data(), (size_t)cap - 1);
            out[cap - 1] = 0;
        }
    }
    return (int)k;
}

// duplex_tag (consensus_helper.py:639-683) on a tag string: the barcode's halves swapped around its
// first '.' (else at len // 2), field 8 R1 -> R2, anything else -> R1.  Fewer than 9 fields is the
// reference's IndexError (-1).  Returns the length (snprintf: the full length even when cap is short).
int ccio_duplex_tag(const char* tag, char* out, int cap) {
    if (!tag) { set_err("duplex_tag: NULL tag"); return -1; }
    auto f = py_split(std::string(tag), '_');
    if (f.size() < 9) { set_err("IndexError in duplex_tag: fewer than 9 fields"); return -1; }
    const std::string bc = f[0];
    const size_t dot = bc.find('.');
    if (dot != std::string::npos) f[0] = bc.substr(dot + 1) + "." + bc.substr(0, dot);
    else f[0] = bc.substr(bc.size() / 2) + bc.substr(0, bc.size() / 2);
    f[8] = f[8] == "R1" ? "R2" : "R1";
    std::string r = f[0];
    for (size_t i = 1; i < f.size(); ++i) r += "_" + f[i];
    return snprintf(out, cap, "%s", r.c_str());
}

int64_t ccio_format_dcs_names(ccio_bam* b, int64_t n, const int64_t* rec_tag, const int64_t* rec_ds, char* blob,
                              int64_t cap, int64_t* off) {
    // lengths in parallel, offsets by a scan, then the names written in parallel straight into the
    // blob (blob NULL: sizes only)
    std::atomic<bool> bad(false);
    const int T = hw_threads(0);
    auto name = [&](int64_t i, char* dst) -> int64_t {
        const uint8_t* ra = b->data.data() + b->rec_off[rec_tag[i]] + 4;
        const uint8_t* rb = b->data.data() + b->rec_off[rec_ds[i]] + 4;
        const size_t la = ra[8] ? (size_t)ra[8] - 1 : 0, lb = rb[8] ? (size_t)rb[8] - 1 : 0;   // l_read_name - NUL
        return dcs_name_into((const char*)ra + 32, la, (const char*)rb + 32, lb, dst);
    };
    parallel_chunks(n, T, 16384, [&](int64_t b0, int64_t e0) {
        for (int64_t i = b0; i < e0 && !bad; ++i) {
            const int64_t k = name(i, nullptr);
            if (k < 0) bad = true;
            else off[i] = k;
        }
    });
    if (bad) { set_err("IndexError in dcs_consensus_tag"); return -1; }
    int64_t used = 0;
    for (int64_t i = 0; i < n; ++i) { const int64_t l = off[i]; off[i] = used; used += l; }
    off[n] = used;
    if (!blob) return used;
    if (used > cap) { set_err("name blob too small"); return -1; }
    parallel_chunks(n, T, 16384, [&](int64_t b0, int64_t e0) {
        for (int64_t i = b0; i < e0; ++i) name(i, blob + off[i]);
    });
    return used;
}

}  // extern "C"

namespace {

int index_stream(const uint8_t* dp, size_t dn, const std::vector<uint64_t>& bco, const std::vector<uint64_t>& buo,
                 const char* path);

inline uint64_t coord_key(const uint8_t* r) {   // r: record core (after block_size)
    const uint64_t tid = (uint32_t)rd32(r), pos = (uint32_t)(rd32(r + 4) + 1);
    return (tid << 32) | (pos << 1) | ((rdu16(r + 14) >> 4) & 1u);
}

// Stable sort of (key, index) items by key: chunks sorted in parallel, then merged pairwise in
// parallel rounds (std::merge takes the left run first on ties, so the order stays stable).
void parallel_stable_sort(std::vector<std::pair<uint64_t, int64_t>>& k, int T) {
    using KV = std::pair<uint64_t, int64_t>;
    auto less = [](const KV& a, const KV& c) { return a.first < c.first; };
    const int64_t n = (int64_t)k.size();
    int parts = 1;
    while (parts < T && n / (parts * 2) >= 65536) parts *= 2;
    std::vector<int64_t> cut(parts + 1);
    for (int i = 0; i <= parts; ++i) cut[i] = n * i / parts;
    parallel_chunks(parts, parts, 1, [&](int64_t b, int64_t) { std::stable_sort(k.begin() + cut[b], k.begin() + cut[b + 1], less); });
    std::vector<KV> tmp(parts > 1 ? n : 0);
    std::vector<KV>* src = &k;
    std::vector<KV>* dst = &tmp;
    for (int w = 1; w < parts; w *= 2) {
        parallel_chunks(parts / (2 * w), parts / (2 * w), 1, [&](int64_t b, int64_t) {
            const int64_t lo = cut[2 * w * b], mid = cut[2 * w * b + w], hi = cut[2 * w * b + 2 * w];
            std::merge(src->begin() + lo, src->begin() + mid, src->begin() + mid, src->begin() + hi, dst->begin() + lo, less);
        });
        std::swap(src, dst);
    }
    if (src != &k) k.swap(*src);
}

// records (raw, block_size first) stably ordered by the samtools-sort stand-in key
void sort_records(std::vector<const uint8_t*>& recs, int T) {
    const int64_t n = (int64_t)recs.size();
    std::vector<std::pair<uint64_t, int64_t>> k(n);
    parallel_chunks(n, T, 65536, [&](int64_t s, int64_t e) {
        for (int64_t i = s; i < e; ++i) k[i] = {coord_key(recs[i] + 4), i};
    });
    parallel_stable_sort(k, T);
    std::vector<const uint8_t*> out(n);
    parallel_chunks(n, T, 65536, [&](int64_t s, int64_t e) {
        for (int64_t i = s; i < e; ++i) out[i] = recs[k[i].second];
    });
    recs.swap(out);
}

// The output of every writer: hdr's header then the records `recs` (raw, block_size first)
// gathered in parallel into one stream, BGZF-written to path.  flags & CCIO_W_INDEX also writes
// path.bai from the stream in memory (samtools index; the member offsets come from the write), and
// keep (non-null) receives a handle over the written stream, as ccio_bam_open would return it.
int finish_stream(const char* path, const ccio_bam* hdr, Bytes&& all, const std::vector<uint64_t>& at, int level,
                  int T, int flags, ccio_bam** keep);

int finish_output(const char* path, const ccio_bam* hdr, const std::vector<const uint8_t*>& recs, int level, int T,
                  int flags, ccio_bam** keep) {
    PhaseTimer pt;
    const int64_t n = (int64_t)recs.size();
    std::vector<uint64_t> at(n + 1);
    at[0] = hdr->header_raw.size();
    {
        // record sizes in parallel chunks, then the chunk sums' prefix, then the offsets
        const int64_t nc = std::max<int64_t>(1, std::min<int64_t>(4 * (int64_t)T, n / 65536 + 1));
        std::vector<uint64_t> csum(nc + 1, 0);
        parallel_for(nc, T, [&](int64_t b, int64_t e, int) {
            for (int64_t c = b; c < e; ++c) {
                const int64_t i0 = n * c / nc, i1 = n * (c + 1) / nc;
                uint64_t acc = 0;
                for (int64_t i = i0; i < i1; ++i) {
                    acc += 4 + (uint64_t)rd32(recs[i]);
                    at[i + 1] = acc;
                }
                csum[c + 1] = acc;
            }
        });
        for (int64_t c = 0; c < nc; ++c) csum[c + 1] += csum[c];
        parallel_for(nc, T, [&](int64_t b, int64_t e, int) {
            for (int64_t c = b; c < e; ++c) {
                const int64_t i0 = n * c / nc, i1 = n * (c + 1) / nc;
                const uint64_t base = at[0] + csum[c];
                for (int64_t i = i0; i < i1; ++i) at[i + 1] += base;
            }
        });
    }
    Bytes all;
    all.resize(at[n]);
    memcpy(all.data(), hdr->header_raw.data(), hdr->header_raw.size());
    parallel_chunks(n, T, 8192, [&](int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) memcpy(all.data() + at[i], recs[i], at[i + 1] - at[i]);
    });
    pt.lap("finish: offsets + copy");
    return finish_stream(path, hdr, std::move(all), at, level, T, flags, keep);
}

// The stream `all` (hdr's header, then the records at offsets at[0..n)) BGZF-written to path, with
// path.bai (CCIO_W_INDEX) and a kept handle (keep non-null) owning the stream.
// BGZF-write the stream [dp, dp + dn) to path, and path.bai (CCIO_W_INDEX)
int write_stream_file(const std::string& path, const uint8_t* dp, size_t dn, int level, int T, int flags) {
    PhaseTimer pt;
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) { set_err("cannot write " + path); return -1; }
    std::vector<uint64_t> cs;
    const bool ok = bgzf_deflate_write(f, dp, dn, level, T, (flags & CCIO_W_INDEX) ? &cs : nullptr);
    if (fclose(f) != 0 || !ok) { set_err("BGZF write failed: " + path); return -1; }
    pt.lap("finish: deflate + write");
    if (flags & CCIO_W_INDEX) {
        std::vector<uint64_t> bco, buo;
        uint64_t off = 0;
        for (size_t i = 0; i < cs.size(); ++i) {
            bco.push_back(off);
            buo.push_back((uint64_t)i * 0xff00);
            off += cs[i];
        }
        bco.push_back(off);
        buo.push_back(dn);
        if (index_stream(dp, dn, bco, buo, path.c_str()) != 0) return -1;
        pt.lap("finish: index");
    }
    return 0;
}

int finish_stream(const char* path, const ccio_bam* hdr, Bytes&& all, const std::vector<uint64_t>& at, int level,
                  int T, int flags, ccio_bam** keep) {
    wait_path(path);   // an earlier asynchronous write of the same file
    std::unique_ptr<ccio_bam> nb;
    if (keep) {
        nb.reset(new ccio_bam());
        nb->header_text = hdr->header_text;
        nb->refs = hdr->refs;
        nb->header_raw = hdr->header_raw;
        nb->rec_off.assign(at.begin(), at.end() - 1);
        nb->data = std::move(all);
    }
    if (!(flags & CCIO_W_ASYNC)) {
        const Bytes& d = nb ? nb->data : all;
        if (write_stream_file(path, d.data(), d.size(), level, T, flags) != 0) return -1;
        if (keep) *keep = nb.release();
        return 0;
    }
    // asynchronous: compressed and written by a thread of its own; the kept handle (which owns the
    // stream) waits for it before it is freed, otherwise the thread owns the stream
    std::shared_ptr<Bytes> own;
    if (!nb) own = std::make_shared<Bytes>(std::move(all));
    const uint8_t* dp = nb ? nb->data.data() : own->data();
    const size_t dn = nb ? nb->data.size() : own->size();
    auto err = std::make_shared<std::string>();
    const std::string p = abs_path(path);
    std::shared_future<int> fut = std::async(std::launch::async, [p, dp, dn, level, T, flags, err, own]() {
                                      const int rc = write_stream_file(p, dp, dn, level, T, flags);
                                      if (rc != 0) *err = g_err;
                                      return rc;
                                  }).share();
    {
        std::lock_guard<std::mutex> lk(g_pend_mu);
        g_pend.push_back({p, fut, err});
    }
    if (keep) {
        nb->pending = fut;
        *keep = nb.release();
    }
    return 0;
}

// Merge of coordinate-sorted record sets (samtools merge stand-in): ties keep input order.  Sorted
// inputs merge in one linear pass (a k-way merge by (key, input)); an input that is not sorted sends
// the whole merge through the stable sort by (key, input, record), the same order.
std::vector<const uint8_t*> merge_order(const std::vector<const ccio_bam*>& bs, int T) {
    const int nin = (int)bs.size();
    std::vector<std::vector<uint64_t>> keys(nin);
    bool sorted = true;
    int64_t total = 0;
    for (int fi = 0; fi < nin; ++fi) {
        const ccio_bam* b = bs[fi];
        const int64_t n = (int64_t)b->rec_off.size();
        keys[fi].resize(n);
        parallel_chunks(n, T, 65536, [&](int64_t s, int64_t e) {
            for (int64_t i = s; i < e; ++i) keys[fi][i] = coord_key(b->data.data() + b->rec_off[i] + 4);
        });
        sorted = sorted && std::is_sorted(keys[fi].begin(), keys[fi].end());
        total += n;
    }
    std::vector<const uint8_t*> recs;
    recs.reserve(total);
    if (sorted) {
        std::vector<int64_t> at(nin, 0);
        for (int64_t o = 0; o < total; ++o) {
            int best = -1;
            for (int fi = 0; fi < nin; ++fi)
                if (at[fi] < (int64_t)keys[fi].size() && (best < 0 || keys[fi][at[fi]] < keys[best][at[best]])) best = fi;
            recs.push_back(bs[best]->data.data() + bs[best]->rec_off[at[best]++]);
        }
    } else {
        struct K { uint64_t key; int f; int64_t i; };
        std::vector<K> k;
        k.reserve(total);
        for (int fi = 0; fi < nin; ++fi)
            for (int64_t i = 0; i < (int64_t)keys[fi].size(); ++i) k.push_back({keys[fi][i], fi, i});
        std::stable_sort(k.begin(), k.end(), [](const K& a, const K& c) {
            if (a.key != c.key) return a.key < c.key;
            return a.f < c.f;
        });
        for (auto& x : k) recs.push_back(bs[x.f]->data.data() + bs[x.f]->rec_off[x.i]);
    }
    return recs;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ writing
// Assemble output records (see cc_out_spec in the header) and write a BGZF BAM
// whose header is copied from `tmpl` (pysam AlignmentFile(..., template=bam)).
int ccio_write_bam(const char* path, ccio_bam* tmpl, ccio_interner* it, int64_t n, const cc_out_spec* spec,
                   ccio_bam* const* srcs, int nsrc, const char* names, const int64_t* name_off,
                   const uint8_t* cons_seq, const uint8_t* cons_qual, int level, int nthreads) {
    return ccio_write_bam_ex(path, tmpl, it, n, spec, srcs, nsrc, names, name_off, cons_seq, cons_qual, level, nthreads,
                             0, nullptr);
}

// ccio_write_bam with flags: CCIO_W_SORT writes the records in samtools-sort order (stable: ties
// keep the spec order), CCIO_W_INDEX also writes path.bai; keep (non-null) receives a handle over
// the written file's records (the next stage reads them without inflating the file again).
int ccio_write_bam_ex(const char* path, ccio_bam* tmpl, ccio_interner* it, int64_t n, const cc_out_spec* spec,
                      ccio_bam* const* srcs, int nsrc, const char* names, const int64_t* name_off,
                      const uint8_t* cons_seq, const uint8_t* cons_qual, int level, int nthreads, int flags,
                      ccio_bam** keep) {
    if (keep) *keep = nullptr;
    PhaseTimer pt;
    const int T = hw_threads(nthreads);
    for (int64_t i = 0; i < n; ++i)
        if (spec[i].src_file < 0 || spec[i].src_file >= nsrc) { set_err("bad output spec"); return -1; }
    const std::vector<std::string>& rgs = it->t[2].strs;
    auto name_of = [&](const cc_out_spec& sp, const char** nm) -> size_t {
        *nm = "";
        if (sp.name_id < 0) return 0;
        *nm = names + name_off[sp.name_id];
        return (size_t)(name_off[sp.name_id + 1] - name_off[sp.name_id]);
    };
    // 1. every record's size (block_size included) and, for a sorted output, its coordinate key
    //    (the output record's tid, pos and reverse bit: the template's, the spec's flag for kind 2)
    std::vector<uint64_t> sz(n);
    const bool sorted = (flags & CCIO_W_SORT) != 0;
    std::vector<std::pair<uint64_t, int64_t>> k(sorted ? n : 0);
    parallel_chunks(n, T, 16384, [&](int64_t s0, int64_t e0) {
        for (int64_t i = s0; i < e0; ++i) {
            const cc_out_spec& sp = spec[i];
            const ccio_bam* src = srcs[sp.src_file];
            const uint8_t* rec = src->data.data() + src->rec_off[sp.src_rec];
            const int32_t bs = rd32(rec);
            const uint8_t* r = rec + 4;
            const char* nm;
            const size_t nl = name_of(sp, &nm);
            const uint8_t lqn = r[8];
            const uint16_t ncig = rdu16(r + 12);
            if (sp.kind == CC_OUT_RAW) sz[i] = 4 + (uint64_t)bs;
            else if (sp.kind == CC_OUT_RENAME) sz[i] = 4 + 32 + nl + 1 + (uint64_t)(bs - 32 - lqn);
            else
                sz[i] = 4 + 32 + nl + 1 + 4 * (uint64_t)ncig + (uint64_t)(sp.cons_len + 1) / 2 + (uint64_t)sp.cons_len +
                        (sp.rg_id >= 0 ? 3 + rgs.at(sp.rg_id).size() + 1 : 0);
            if (sorted) {
                const uint64_t tid = (uint32_t)rd32(r), pos = (uint32_t)(rd32(r + 4) + 1);
                const uint32_t fl = sp.kind == CC_OUT_NEW ? (uint32_t)(uint16_t)sp.flag : rdu16(r + 14);
                k[i] = {(tid << 32) | (pos << 1) | ((fl >> 4) & 1u), i};
            }
        }
    });
    if (sorted) parallel_stable_sort(k, T);   // samtools sort order, ties in spec order
    pt.lap("write: sizes + sort");
    // 2. offsets in output order, then every record assembled in place
    std::vector<uint64_t> at(n + 1);
    at[0] = tmpl->header_raw.size();
    {
        const int64_t nc = std::max<int64_t>(1, std::min<int64_t>(4 * (int64_t)T, n / 65536 + 1));
        std::vector<uint64_t> csum(nc + 1, 0);
        parallel_for(nc, T, [&](int64_t b0, int64_t e0, int) {
            for (int64_t c = b0; c < e0; ++c) {
                const int64_t i0 = n * c / nc, i1 = n * (c + 1) / nc;
                uint64_t acc = 0;
                for (int64_t o = i0; o < i1; ++o) {
                    acc += sz[sorted ? k[o].second : o];
                    at[o + 1] = acc;
                }
                csum[c + 1] = acc;
            }
        });
        for (int64_t c = 0; c < nc; ++c) csum[c + 1] += csum[c];
        parallel_for(nc, T, [&](int64_t b0, int64_t e0, int) {
            for (int64_t c = b0; c < e0; ++c) {
                const int64_t i0 = n * c / nc, i1 = n * (c + 1) / nc;
                const uint64_t base = at[0] + csum[c];
                for (int64_t o = i0; o < i1; ++o) at[o + 1] += base;
            }
        });
    }
    Bytes all;
    all.resize(at[n]);
    memcpy(all.data(), tmpl->header_raw.data(), tmpl->header_raw.size());
    parallel_chunks(n, T, 8192, [&](int64_t s0, int64_t e0) {
        for (int64_t o = s0; o < e0; ++o) {
            const cc_out_spec& sp = spec[sorted ? k[o].second : o];
            const ccio_bam* src = srcs[sp.src_file];
            const uint8_t* rec = src->data.data() + src->rec_off[sp.src_rec];
            const int32_t bs = rd32(rec);
            const uint8_t* r = rec + 4;
            uint8_t* d = all.data() + at[o];
            auto put = [&](const void* p, size_t len) { memcpy(d, p, len); d += len; };
            auto put32 = [&](int32_t v) { put(&v, 4); };
            auto put16 = [&](uint16_t v) { put(&v, 2); };
            if (sp.kind == CC_OUT_RAW) { put(rec, 4 + (size_t)bs); continue; }
            const char* nm;
            const size_t nl = name_of(sp, &nm);
            const uint8_t lqn = r[8];
            const uint16_t ncig = rdu16(r + 12);
            if (sp.kind == CC_OUT_RENAME) {
                // qname replaced, everything else byte-identical
                put32((int32_t)(32 + nl + 1 + (size_t)(bs - 32 - lqn)));
                uint8_t* core = d;
                put(r, 32);
                core[8] = (uint8_t)(nl + 1);
                put(nm, nl);
                *d++ = 0;
                put(r + 32 + lqn, (size_t)(bs - 32 - lqn));
                continue;
            }
            // CC_OUT_NEW: create_aligned_segment (consensus_helper.py:568-619)
            const int32_t L = sp.cons_len;
            const uint8_t* cg = r + 32 + lqn;
            const int64_t pos = rd32(r + 4);
            int64_t rlen = 0;
            for (int c = 0; c < ncig; ++c) {
                const uint32_t v = rdu32(cg + 4 * c), op = v & 0xf;
                if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rlen += v >> 4;
            }
            const int64_t endp = pos + (rlen ? rlen : 1);
            const int bin = reg2bin(pos < 0 ? 0 : pos, pos < 0 ? 1 : endp);
            const std::string* rgv = sp.rg_id >= 0 ? &rgs.at(sp.rg_id) : nullptr;
            put32((int32_t)(at[o + 1] - at[o] - 4));
            put32(rd32(r + 0));                 // reference_id (template)
            put32((int32_t)pos);                // reference_start (template)
            *d++ = (uint8_t)(nl + 1);
            *d++ = (uint8_t)sp.mapq;
            put16((uint16_t)bin);
            put16(ncig);
            put16((uint16_t)sp.flag);
            put32(L);
            put32(rd32(r + 20));                // next_reference_id
            put32(rd32(r + 24));                // next_reference_start
            put32(sp.tlen);
            put(nm, nl);
            *d++ = 0;
            put(cg, 4 * (size_t)ncig);
            put(cons_seq + sp.cons_off / 2, (size_t)(L + 1) / 2);
            put(cons_qual + sp.cons_off, (size_t)L);
            if (rgv) {
                put("RGZ", 3);
                put(rgv->data(), rgv->size());
                *d++ = 0;
            }
        }
    });
    pt.lap("write: assemble");
    return finish_stream(path, tmpl, std::move(all), at, level, T, flags, keep);
}


// Stable coordinate sort of a BAM (samtools sort stand-in, ConsensusCruncher.py:10-34):
// key = tid<<32 | (pos+1)<<1 | is_reverse on unsigned tid (unmapped tid -1 last).
int ccio_sort_bam(const char* in_path, const char* out_path, int level, int nthreads) {
    return ccio_sort_bam_ex(in_path, out_path, level, nthreads, 0);
}

// ccio_sort_bam with flags (CCIO_W_INDEX: also out_path.bai)
int ccio_sort_bam_ex(const char* in_path, const char* out_path, int level, int nthreads, int flags) {
    wait_path(in_path);
    const int T = hw_threads(nthreads);
    std::unique_ptr<ccio_bam> b(ccio_bam_open(in_path, nthreads));
    if (!b) return -1;
    std::vector<const uint8_t*> recs(b->rec_off.size());
    for (size_t i = 0; i < recs.size(); ++i) recs[i] = b->data.data() + b->rec_off[i];
    sort_records(recs, T);
    return finish_output(out_path, b.get(), recs, level, T, flags & CCIO_W_INDEX, nullptr);
}

int ccio_merge_bams(const char* out_path, const char* const* in_paths, int nin, int level, int nthreads) {
    for (int i = 0; i < nin; ++i) wait_path(in_paths[i]);
    std::vector<ccio_bam*> bs;
    for (int i = 0; i < nin; ++i) {
        ccio_bam* b = ccio_bam_open(in_paths[i], nthreads);
        if (!b) { for (auto x : bs) ccio_bam_close(x); return -1; }
        bs.push_back(b);
    }
    const int rc = ccio_merge_handles(out_path, bs.data(), nin, level, nthreads, 0, nullptr);
    for (auto x : bs) ccio_bam_close(x);
    return rc;
}

// Merge of coordinate-sorted BAMs held in memory (samtools merge stand-in, ties keep input order;
// the first input's header), with the writer flags (CCIO_W_INDEX) and an optional kept handle.
int ccio_merge_handles(const char* out_path, ccio_bam* const* ins, int nin, int level, int nthreads, int flags,
                       ccio_bam** keep) {
    if (keep) *keep = nullptr;
    if (nin < 1) { set_err("merge: no input"); return -1; }
    const int T = hw_threads(nthreads);
    std::vector<const ccio_bam*> bs(ins, ins + nin);
    const std::vector<const uint8_t*> recs = merge_order(bs, T);
    return finish_output(out_path, bs[0], recs, level, T, flags & (CCIO_W_INDEX | CCIO_W_ASYNC), keep);
}

// Records of several BAM files in file order, one after the other (the first file's header): the
// parts of a sharded stage output joined in rank order (consensuscruncher_amd/sharded.py).
int ccio_concat_bams(const char* out_path, const char* const* in_paths, int nin, int level, int nthreads) {
    for (int i = 0; i < nin; ++i) wait_path(in_paths[i]);
    if (nin < 1) { set_err("concat: no input"); return -1; }
    FILE* f = fopen(out_path, "wb");
    if (!f) { set_err("concat: cannot write"); return -1; }
    // each part is inflated and deflated on its own (BGZF members need not align with records), so
    // peak memory is one part, not the whole output
    bool ok = true;
    for (int i = 0; i < nin && ok; ++i) {
        ccio_bam* b = ccio_bam_open(in_paths[i], nthreads);
        if (!b) { fclose(f); return -1; }
        const uint8_t* beg = b->rec_off.empty() ? b->data.data() + b->data.size() : b->data.data() + b->rec_off[0];
        const size_t nrec = (size_t)(b->data.data() + b->data.size() - beg);
        if (i == 0) ok = bgzf_deflate_blocks(f, b->header_raw.data(), b->header_raw.size(), level, 1);
        ok = ok && bgzf_deflate_blocks(f, beg, nrec, level, hw_threads(nthreads));
        ccio_bam_close(b);
    }
    ok = ok && fwrite(kBgzfEof, 1, 28, f) == 28;
    fclose(f);
    if (!ok) { set_err("concat write failed"); return -1; }
    return 0;
}

// BAI index of a coordinate-sorted BAM (what `samtools index` writes next to the sorted files,
// ConsensusCruncher.py:10-34): per reference the bins with their chunks of virtual file offsets
// (compressed block offset << 16 | offset in the block), the 16 kbp linear index, htslib's
// metadata pseudo-bin 37450 (the reference's offset span, mapped / unmapped counts), and the count
// of records without coordinates.  Written to <path>.bai.
}  // extern "C"

namespace {
// The BAI of one coordinate-sorted BAM stream held in memory (data: the whole uncompressed
// stream from the magic on; bco / buo: per non-empty BGZF member its compressed offset and
// uncompressed start, then the EOF member's offset and the stream's length), written to path.bai.
int index_stream(const uint8_t* dp, size_t dn, const std::vector<uint64_t>& bco, const std::vector<uint64_t>& buo,
                 const char* path) {
    struct Span {
        const uint8_t* p; size_t n;
        size_t size() const { return n; }
        const uint8_t* data() const { return p; }
        const uint8_t& operator[](size_t i) const { return p[i]; }
    } data{dp, dn};
    // the records come in stream order: the member holding an offset is found by walking forward
    // from the previous one (amortised O(1), not a search per record)
    size_t vcur = 0;
    auto voff = [&](uint64_t u) {
        if (u < buo[vcur]) vcur = std::upper_bound(buo.begin(), buo.end(), u) - buo.begin() - 1;
        while (vcur + 1 < buo.size() && buo[vcur + 1] <= u) ++vcur;
        return (bco[vcur] << 16) | (u - buo[vcur]);
    };
    if (data.size() < 12 || memcmp(data.data(), "BAM\1", 4) != 0) { set_err("index: not a BAM file"); return -1; }
    size_t off = 4;
    const int32_t ltext = rd32(&data[off]);
    if (ltext < 0 || off + 8 + (size_t)ltext > data.size()) { set_err("index: truncated header"); return -1; }
    off += 4 + ltext;
    const int32_t nref = rd32(&data[off]);
    off += 4;
    if (nref < 0) { set_err("index: bad reference count"); return -1; }
    for (int32_t i = 0; i < nref; ++i) {
        if (off + 4 > data.size()) { set_err("index: truncated header"); return -1; }
        const int32_t ln = rd32(&data[off]);
        if (ln < 0 || off + 8 + (size_t)ln > data.size()) { set_err("index: truncated header"); return -1; }
        off += 4 + ln + 4;
    }
    struct Ref {
        std::map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>> bins;
        std::vector<uint64_t> lin;
        uint64_t beg = ~0ULL, end = 0, mapped = 0, unmapped = 0;
    };
    std::vector<Ref> refs(nref);
    uint64_t no_coor = 0;
    // the last bin touched (sorted records mostly land in the bin of the record before them)
    int32_t cache_tid = -1;
    uint32_t cache_bin = 0;
    std::vector<std::pair<uint64_t, uint64_t>>* cache_ch = nullptr;
    int32_t last_tid = -2;
    int64_t last_pos = -1;
    while (off + 4 <= data.size()) {
        const int32_t bs = rd32(&data[off]);
        if (bs < 32 || off + 4 + (size_t)bs > data.size()) { set_err("index: truncated BAM record"); return -1; }
        const uint8_t* r = &data[off + 4];
        const int32_t tid = rd32(r), pos = rd32(r + 4);
        const uint16_t ncig = rdu16(r + 12), flag = rdu16(r + 14);
        if (32 + (size_t)r[8] + 4 * (size_t)ncig > (size_t)bs) { set_err("index: record cigar past its end"); return -1; }
        const uint64_t vb = voff(off), ve = voff(off + 4 + bs);
        if ((tid >= 0 && tid < last_tid) || (tid == last_tid && pos < last_pos) || (tid >= 0 && last_tid == -1)) {
            set_err("index: BAM not coordinate-sorted");
            return -1;
        }
        last_tid = tid;
        last_pos = pos;
        off += 4 + bs;
        if (tid < 0 || tid >= nref) { ++no_coor; continue; }
        int64_t rl = 0;
        if (!(flag & 4)) {
            const uint8_t* cg = r + 32 + r[8];
            for (int c = 0; c < ncig; ++c) {
                const uint32_t v = rdu32(cg + 4 * c), op = v & 0xf;
                if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += v >> 4;
            }
        }
        const int64_t beg = pos < 0 ? 0 : pos, end = beg + (rl ? rl : 1);
        Ref& R = refs[tid];
        const uint32_t bin = (uint32_t)reg2bin(beg, end);
        if (!cache_ch || cache_tid != tid || cache_bin != bin) {
            cache_ch = &R.bins[bin];   // std::map: the pointer stays valid as bins are added
            cache_tid = tid;
            cache_bin = bin;
        }
        auto& ch = *cache_ch;
        if (!ch.empty() && ch.back().second == vb) ch.back().second = ve;
        else ch.push_back({vb, ve});
        const int64_t w0 = beg >> 14, w1 = (end - 1) >> 14;
        if ((int64_t)R.lin.size() <= w1) R.lin.resize(w1 + 1, 0);
        for (int64_t w = w0; w <= w1; ++w)
            if (!R.lin[w]) R.lin[w] = vb;
        R.beg = std::min(R.beg, vb);
        R.end = std::max(R.end, ve);
        if (flag & 4) ++R.unmapped;
        else ++R.mapped;
    }
    std::string out("BAI\1", 4);
    wr32(out, nref);
    auto w64 = [&](uint64_t v) { out.append((const char*)&v, 8); };
    for (Ref& R : refs) {
        const bool any = R.mapped + R.unmapped > 0;
        wr32(out, (int32_t)R.bins.size() + (any ? 1 : 0));
        for (auto& b : R.bins) {
            wr32(out, (int32_t)b.first);
            wr32(out, (int32_t)b.second.size());
            for (auto& c : b.second) { w64(c.first); w64(c.second); }
        }
        if (any) {   // htslib's metadata pseudo-bin
            wr32(out, 37450);
            wr32(out, 2);
            w64(R.beg); w64(R.end); w64(R.mapped); w64(R.unmapped);
        }
        for (size_t w = 1; w < R.lin.size(); ++w)
            if (!R.lin[w]) R.lin[w] = R.lin[w - 1];
        wr32(out, (int32_t)R.lin.size());
        for (uint64_t v : R.lin) w64(v);
    }
    w64(no_coor);
    const std::string ipath = std::string(path) + ".bai";
    FILE* g = fopen(ipath.c_str(), "wb");
    if (!g || fwrite(out.data(), 1, out.size(), g) != out.size()) {
        if (g) fclose(g);
        set_err("cannot write " + ipath);
        return -1;
    }
    fclose(g);
    return 0;
}

}  // namespace

extern "C" {

int ccio_index_bam(const char* path) {
    wait_path(path);
    FILE* f = fopen(path, "rb");
    if (!f) { set_err(std::string("cannot open ") + path); return -1; }
    std::vector<uint8_t> comp;
    {
        uint8_t buf[1 << 16];
        size_t k;
        while ((k = fread(buf, 1, sizeof buf, f)) > 0) comp.insert(comp.end(), buf, buf + k);
        fclose(f);
    }
    std::vector<uint64_t> bco, buo;   // per block: compressed offset, uncompressed start
    {
        size_t off = 0, u = 0;
        while (off + 18 <= comp.size()) {
            const uint8_t* p = comp.data() + off;
            const uint16_t xlen = p[10] | (p[11] << 8);
            if (off + 12 + (size_t)xlen > comp.size()) { set_err("index: truncated BGZF header"); return -1; }
            size_t bsize = 0;
            for (size_t x = 12; x + 4 <= 12 + (size_t)xlen;) {
                const uint16_t slen = p[x + 2] | (p[x + 3] << 8);
                if (p[x] == 66 && p[x + 1] == 67 && slen == 2 && x + 6 <= 12 + (size_t)xlen)
                    bsize = (size_t)(p[x + 4] | (p[x + 5] << 8)) + 1;
                x += 4 + slen;
            }
            if (!bsize || bsize < 12 + (size_t)xlen + 8 || off + bsize > comp.size()) {
                set_err("index: bad BGZF block");
                return -1;
            }
            const uint8_t* t = p + bsize - 4;
            const size_t isize = (size_t)t[0] | ((size_t)t[1] << 8) | ((size_t)t[2] << 16) | ((size_t)t[3] << 24);
            if (isize) { bco.push_back(off); buo.push_back(u); }
            u += isize;
            off += bsize;
        }
        bco.push_back(off);   // the EOF block: the offset just past the data
        buo.push_back(u);
    }
    Bytes data;
    std::string err;
    if (!bgzf_inflate_all(comp, data, hw_threads(0), err)) { set_err(err); return -1; }
    return index_stream(data.data(), data.size(), bco, buo, path);
}

// ------------------------------------------------------------------ rank-local record sets
// The multi-GPU driver (consensuscruncher_amd/sharded.py) keeps on each rank only the records of its
// block of bed regions: read through the BAI (the regions' BGZF blocks only), completed by records
// other ranks send (raw BAM records), sorted and merged in memory.  These handles behave like
// ccio_bam_open's (decode, write, names).
}  // extern "C"

namespace {

struct BaiRef {
    std::map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>> bins;
    std::vector<uint64_t> lin;
    uint64_t first = ~0ULL;   // the reference's first record (smallest chunk start)
    // the first record that can start at or after b0 (linear-index windows before the reference's
    // first record hold 0)
    uint64_t start(int64_t b0) const { return std::max(lin[(size_t)(b0 >> 14)], first); }
};

bool read_bai(const std::string& path, std::vector<BaiRef>& refs, std::string& err) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open " + path + " (index the BAM first)"; return false; }
    std::vector<uint8_t> d;
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + k);
    fclose(f);
    size_t o = 0;
    auto need = [&](size_t n) { return o + n <= d.size(); };
    if (!need(8) || memcmp(d.data(), "BAI\1", 4) != 0) { err = "not a BAI index: " + path; return false; }
    o = 4;
    const int32_t nref = rd32(&d[o]);
    o += 4;
    refs.assign(nref > 0 ? nref : 0, BaiRef());
    for (int32_t r = 0; r < nref; ++r) {
        if (!need(4)) { err = "truncated BAI"; return false; }
        const int32_t nbin = rd32(&d[o]);
        o += 4;
        for (int32_t b = 0; b < nbin; ++b) {
            if (!need(8)) { err = "truncated BAI"; return false; }
            const uint32_t bin = rdu32(&d[o]);
            const int32_t nch = rd32(&d[o + 4]);
            o += 8;
            if (nch < 0 || !need((size_t)nch * 16)) { err = "truncated BAI"; return false; }
            auto& v = refs[r].bins[bin];
            for (int32_t c = 0; c < nch; ++c) {
                uint64_t a, e;
                memcpy(&a, &d[o], 8);
                memcpy(&e, &d[o + 8], 8);
                v.push_back({a, e});
                o += 16;
            }
        }
        if (!need(4)) { err = "truncated BAI"; return false; }
        const int32_t nin = rd32(&d[o]);
        o += 4;
        if (nin < 0 || !need((size_t)nin * 8)) { err = "truncated BAI"; return false; }
        refs[r].lin.resize(nin);
        if (nin) memcpy(refs[r].lin.data(), &d[o], (size_t)nin * 8);
        o += (size_t)nin * 8;
        for (auto& b : refs[r].bins)
            if (b.first != 37450)
                for (auto& c : b.second) refs[r].first = std::min(refs[r].first, c.first);
    }
    return true;
}

// SAM spec reg2bins: the bins that may hold records overlapping [beg, end)
void reg2bins(int64_t beg, int64_t end, std::vector<uint32_t>& out) {
    out.clear();
    --end;
    out.push_back(0);
    const int shifts[5] = {26, 23, 20, 17, 14};
    const uint32_t base[5] = {1, 9, 73, 585, 4681};
    for (int l = 0; l < 5; ++l)
        for (int64_t k = base[l] + (beg >> shifts[l]); k <= (int64_t)base[l] + (end >> shifts[l]); ++k)
            out.push_back((uint32_t)k);
}

// the compressed bytes [a, b) of the file
bool pread_range(int fd, uint64_t a, uint64_t b, std::vector<uint8_t>& out) {
    out.resize(b - a);
    size_t got = 0;
    while (got < out.size()) {
        const ssize_t k = pread(fd, out.data() + got, out.size() - got, (off_t)(a + got));
        if (k <= 0) return false;
        got += (size_t)k;
    }
    return true;
}

// one BGZF member's sizes at p (false if the bytes end before it)
bool bgzf_member(const uint8_t* p, size_t avail, size_t* bsize, size_t* hdr, size_t* isize) {
    if (avail < 18 || p[0] != 0x1f || p[1] != 0x8b) return false;
    const uint16_t xlen = p[10] | (p[11] << 8);
    size_t bs = 0;
    for (size_t x = 12; x + 4 <= 12 + (size_t)xlen && x + 4 <= avail;) {
        const uint16_t slen = p[x + 2] | (p[x + 3] << 8);
        if (p[x] == 66 && p[x + 1] == 67 && slen == 2 && x + 6 <= avail) bs = (size_t)(p[x + 4] | (p[x + 5] << 8)) + 1;
        x += 4 + slen;
    }
    if (!bs || bs > avail) return false;
    const uint8_t* t = p + bs - 4;
    *bsize = bs;
    *hdr = 12 + xlen;
    *isize = (size_t)t[0] | ((size_t)t[1] << 8) | ((size_t)t[2] << 16) | ((size_t)t[3] << 24);
    return true;
}

// Inflates the whole BGZF members of comp (file offset base) in parallel; coff[i] / uoff[i] per member.
template <class Vec>
bool inflate_members(const std::vector<uint8_t>& comp, uint64_t base, Vec& out,
                     std::vector<uint64_t>& coff, std::vector<uint64_t>& uoff, int nthreads, std::string& err) {
    struct Blk { size_t c, clen, u, ulen; };
    std::vector<Blk> bl;
    size_t o = 0, u = 0;
    coff.clear();
    uoff.clear();
    while (o < comp.size()) {
        size_t bs, hd, is;
        if (!bgzf_member(comp.data() + o, comp.size() - o, &bs, &hd, &is)) break;   // a partial member: past the range
        bl.push_back({o + hd, bs - hd - 8, u, is});
        coff.push_back(base + o);
        uoff.push_back(u);
        u += is;
        o += bs;
    }
    coff.push_back(base + o);
    uoff.push_back(u);
    out.resize(u);
    std::atomic<bool> bad(false);
    parallel_chunks((int64_t)bl.size(), nthreads, 16, [&](int64_t b, int64_t e) {
        Codec c;
        for (int64_t i = b; i < e && !bad; ++i) {
            if (!bl[i].ulen) continue;
            if (!c.inflate_raw(comp.data() + bl[i].c, bl[i].clen, out.data() + bl[i].u, bl[i].ulen)) bad = true;
        }
    });
    if (bad) { err = "BGZF inflate failed"; return false; }
    return true;
}

// the header (magic .. refs) of the BAM at fd
bool read_header(int fd, uint64_t fsize, ccio_bam* b, std::string& err) {
    std::vector<uint8_t> comp, data;
    std::vector<uint64_t> co, uo;
    for (uint64_t want = 1 << 20;; want *= 4) {
        const uint64_t e = std::min<uint64_t>(want, fsize);
        if (!pread_range(fd, 0, e, comp)) { err = "short read"; return false; }
        if (!inflate_members(comp, 0, data, co, uo, 1, err)) return false;
        size_t off = 4;
        bool ok = data.size() >= 12 && memcmp(data.data(), "BAM\1", 4) == 0;
        if (ok) {
            const int32_t ltext = rd32(&data[off]);
            off += 4 + (size_t)ltext;
            ok = off + 4 <= data.size();
            if (ok) {
                const int32_t nref = rd32(&data[off]);
                off += 4;
                b->refs.clear();
                for (int32_t i = 0; i < nref && ok; ++i) {
                    if (off + 4 > data.size()) { ok = false; break; }
                    const int32_t ln = rd32(&data[off]);
                    if (off + 8 + (size_t)ln > data.size()) { ok = false; break; }
                    b->refs.emplace_back(std::string((const char*)&data[off + 4], ln > 0 ? ln - 1 : 0),
                                         rd32(&data[off + 4 + ln]));
                    off += 8 + ln;
                }
                if (ok) {
                    b->header_text.assign((const char*)&data[8], strnlen((const char*)&data[8], rd32(&data[4])));
                    b->header_raw.assign(data.begin(), data.begin() + off);
                    return true;
                }
            }
        }
        if (e >= fsize) { err = "not a BAM file (header)"; return false; }
    }
}

inline uint64_t samtools_key(const uint8_t* r) {   // r: record core (after block_size)
    const uint64_t tid = (uint32_t)rd32(r), pos = (uint32_t)(rd32(r + 4) + 1);
    return (tid << 32) | (pos << 1) | ((rdu16(r + 14) >> 4) & 1u);
}

// a handle over the records `recs` (raw, block_size first), with b's header
ccio_bam* handle_of(const ccio_bam* hdr, const std::vector<std::pair<const uint8_t*, int64_t>>& recs,
                    const std::vector<int64_t>* origin = nullptr) {
    std::unique_ptr<ccio_bam> nb(new ccio_bam());
    nb->header_text = hdr->header_text;
    nb->refs = hdr->refs;
    nb->header_raw = hdr->header_raw;
    size_t tot = nb->header_raw.size();
    for (auto& r : recs) tot += 4 + (size_t)rd32(r.first);
    nb->data.reserve(tot);
    nb->data.assign(nb->header_raw.begin(), nb->header_raw.end());
    nb->rec_off.reserve(recs.size());
    for (auto& r : recs) {
        nb->rec_off.push_back(nb->data.size());
        nb->data.insert(nb->data.end(), r.first, r.first + 4 + rd32(r.first));
    }
    if (origin) nb->origin = *origin;
    return nb.release();
}

}  // namespace

extern "C" {

// Records of the coordinate-sorted, BAI-indexed BAM at path with tid == tid[i] and beg[i] <= pos <
// end[i] for some region i (pysam's region fetch + consensus_helper.py:391-396), in file order,
// each once.  Only the BGZF blocks the index names for the regions are read and inflated.
ccio_bam* ccio_bam_open_regions(const char* path, int32_t n, const int32_t* tid, const int64_t* beg,
                                const int64_t* end, int nthreads) {
    wait_path(path);
    std::string err;
    std::vector<BaiRef> bai;
    if (!read_bai(std::string(path) + ".bai", bai, err)) { set_err(err); return nullptr; }
    const int fd = open(path, O_RDONLY);
    if (fd < 0) { set_err(std::string("cannot open ") + path); return nullptr; }
    struct stat st;
    fstat(fd, &st);
    const uint64_t fsize = (uint64_t)st.st_size;
    std::unique_ptr<ccio_bam> hb(new ccio_bam());
    if (!read_header(fd, fsize, hb.get(), err)) { close(fd); set_err(err + ": " + path); return nullptr; }
    // per region: the compressed span [first block, last block] its records can lie in
    struct Span { uint64_t v0, c1; int32_t t; int64_t b, e; };
    std::vector<Span> spans;
    std::vector<uint32_t> bins;
    for (int32_t i = 0; i < n; ++i) {
        const int32_t t = tid[i];
        if (t < 0 || t >= (int32_t)bai.size() || end[i] <= beg[i]) continue;
        const BaiRef& R = bai[t];
        if (R.lin.empty()) continue;
        const int64_t b0 = std::max<int64_t>(beg[i], 0);
        if ((size_t)(b0 >> 14) >= R.lin.size() || R.first == ~0ULL) continue;   // no record at or after beg on t
        const uint64_t v0 = R.start(b0);
        uint64_t vmax = 0;
        reg2bins(b0, end[i], bins);
        for (uint32_t bn : bins) {
            auto it = R.bins.find(bn);
            if (it == R.bins.end()) continue;
            for (auto& c : it->second)
                if (c.second > v0) vmax = std::max(vmax, c.second);
        }
        if (vmax <= v0) continue;
        spans.push_back({v0, vmax >> 16, t, b0, end[i]});
    }
    std::sort(spans.begin(), spans.end(), [](const Span& a, const Span& c) { return a.v0 < c.v0; });
    std::vector<std::pair<uint64_t, uint64_t>> picked;   // (voffset, offset of the record in arena)
    std::vector<uint8_t> arena;
    std::vector<uint8_t> comp, data;
    std::vector<uint64_t> co, uo;
    const int T = hw_threads(nthreads);
    for (size_t s0 = 0; s0 < spans.size();) {
        // spans sharing or touching blocks are read together
        uint64_t c0 = spans[s0].v0 >> 16, c1 = spans[s0].c1;
        size_t s1 = s0 + 1;
        while (s1 < spans.size() && (spans[s1].v0 >> 16) <= c1 + 1) { c1 = std::max(c1, spans[s1].c1); ++s1; }
        const uint64_t stop = std::min<uint64_t>(fsize, c1 + 65536 + 64);   // the last block whole
        if (!pread_range(fd, c0, stop, comp)) { close(fd); set_err("short read"); return nullptr; }
        if (!inflate_members(comp, c0, data, co, uo, T, err)) { close(fd); set_err(err); return nullptr; }
        for (size_t s = s0; s < s1; ++s) {
            const Span& sp = spans[s];
            const size_t bi = std::lower_bound(co.begin(), co.end(), sp.v0 >> 16) - co.begin();
            if (bi >= co.size() - 1 || co[bi] != (sp.v0 >> 16)) { close(fd); set_err("index offset not at a block"); return nullptr; }
            size_t u = uo[bi] + (sp.v0 & 0xffff);
            while (u + 4 <= data.size()) {
                const int32_t bs = rd32(&data[u]);
                if (bs < 32 || u + 4 + (size_t)bs > data.size()) break;   // past the span
                const uint8_t* r = &data[u + 4];
                const int32_t t = rd32(r), pos = rd32(r + 4);
                if (t != sp.t || pos >= sp.e) break;
                if (pos >= sp.b) {
                    const size_t b = std::upper_bound(uo.begin(), uo.end(), u) - uo.begin() - 1;
                    const uint64_t v = (co[b] << 16) | (u - uo[b]);
                    picked.emplace_back(v, (uint64_t)arena.size());
                    arena.insert(arena.end(), &data[u], &data[u] + 4 + bs);
                }
                u += 4 + (size_t)bs;
            }
        }
        s0 = s1;
    }
    close(fd);
    std::sort(picked.begin(), picked.end());
    std::vector<std::pair<const uint8_t*, int64_t>> recs;
    for (size_t i = 0; i < picked.size(); ++i)
        if (i == 0 || picked[i].first != picked[i - 1].first) recs.push_back({arena.data() + picked[i].second, 0});
    return handle_of(hb.get(), recs);
}

// per record: tid, pos, mtid, mpos, flag (any may be NULL)
int ccio_bam_cores(ccio_bam* b, int32_t* tid, int32_t* pos, int32_t* mtid, int32_t* mpos, uint16_t* flag) {
    const int64_t n = (int64_t)b->rec_off.size();
    for (int64_t i = 0; i < n; ++i) {
        const uint8_t* r = b->data.data() + b->rec_off[i] + 4;
        if (tid) tid[i] = rd32(r);
        if (pos) pos[i] = rd32(r + 4);
        if (mtid) mtid[i] = rd32(r + 20);
        if (mpos) mpos[i] = rd32(r + 24);
        if (flag) flag[i] = rdu16(r + 14);
    }
    return 0;
}

// the raw records idx[0..n) concatenated (block_size first); out NULL: the size
int64_t ccio_bam_pack(ccio_bam* b, int64_t n, const int64_t* idx, uint8_t* out, int64_t cap) {
    int64_t used = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (idx[i] < 0 || idx[i] >= (int64_t)b->rec_off.size()) { set_err("pack: record index"); return -1; }
        const uint8_t* rec = b->data.data() + b->rec_off[idx[i]];
        const int64_t k = 4 + rd32(rec);
        if (out) {
            if (used + k > cap) { set_err("pack: buffer too small"); return -1; }
            memcpy(out + used, rec, (size_t)k);
        }
        used += k;
    }
    return used;
}

// A handle over the records of parts[0..n) and the raw record blobs[0..nb) (block_size first, as
// ccio_bam_pack writes them), in that order, then stably sorted: key 0 = (tid, pos) with unmapped
// (tid -1) last, 1 = samtools sort's stand-in key (tid, pos, is_reverse; ccio_sort_bam), 2 = none.
// The header is parts[0]'s (or tmpl's).
ccio_bam* ccio_bam_combine(ccio_bam* tmpl, ccio_bam* const* parts, int32_t n, const uint8_t* const* blobs,
                           const int64_t* blob_bytes, int32_t nb, int key, int nthreads) {
    (void)nthreads;
    const ccio_bam* h = tmpl ? tmpl : (n > 0 ? parts[0] : nullptr);
    if (!h) { set_err("combine: no header"); return nullptr; }
    std::vector<std::pair<const uint8_t*, int64_t>> recs;
    for (int32_t p = 0; p < n; ++p)
        for (uint64_t o : parts[p]->rec_off) recs.push_back({parts[p]->data.data() + o, 0});
    for (int32_t k = 0; k < nb; ++k) {
        int64_t o = 0;
        while (o + 4 <= blob_bytes[k]) {
            const int32_t bs = rd32(blobs[k] + o);
            if (bs < 32 || o + 4 + bs > blob_bytes[k]) { set_err("combine: truncated record blob"); return nullptr; }
            recs.push_back({blobs[k] + o, 0});
            o += 4 + bs;
        }
    }
    std::vector<int64_t> origin(recs.size());
    for (size_t i = 0; i < recs.size(); ++i) origin[i] = (int64_t)i;
    if (key != 2) {
        std::vector<std::pair<uint64_t, int64_t>> ks(recs.size());
        for (size_t i = 0; i < recs.size(); ++i) {
            const uint8_t* c = recs[i].first + 4;
            uint64_t k;
            if (key == 0) {
                const uint64_t t = rd32(c) < 0 ? 0xffffffffULL : (uint32_t)rd32(c);
                k = (t << 32) | (uint32_t)rd32(c + 4);
            } else {
                k = samtools_key(c);
            }
            ks[i] = {k, (int64_t)i};
        }
        std::stable_sort(ks.begin(), ks.end(), [](const std::pair<uint64_t, int64_t>& a,
                                                  const std::pair<uint64_t, int64_t>& c) { return a.first < c.first; });
        std::vector<std::pair<const uint8_t*, int64_t>> sorted(recs.size());
        for (size_t i = 0; i < ks.size(); ++i) {
            sorted[i] = recs[ks[i].second];
            origin[i] = ks[i].second;
        }
        recs.swap(sorted);
    }
    return handle_of(h, recs, &origin);
}
// each record's index in the inputs of the ccio_bam_combine that made b (out[nrec]); -1: none
int ccio_bam_origin(ccio_bam* b, int64_t* out) {
    if (b->origin.size() != b->rec_off.size()) { set_err("not a combined handle"); return -1; }
    memcpy(out, b->origin.data(), sizeof(int64_t) * b->origin.size());
    return 0;
}

// the records of b as a BGZF BAM at path (b's header)
int ccio_bam_write_all(const char* path, ccio_bam* b, int level, int nthreads) {
    FILE* f = fopen(path, "wb");
    if (!f) { set_err(std::string("cannot write ") + path); return -1; }
    const bool ok = bgzf_deflate_write(f, b->data.data(), b->data.size(), level, hw_threads(nthreads));
    fclose(f);
    if (!ok) { set_err("BGZF write failed"); return -1; }
    return 0;
}

// the mapped / unmapped counts of the BAI's pseudo-bins summed over the references (pysam's
// AlignmentFile.mapped); -1 when the index has none
int64_t ccio_bai_mapped(const char* path) {
    wait_path(path);
    std::vector<BaiRef> bai;
    std::string err;
    if (!read_bai(std::string(path) + ".bai", bai, err)) { set_err(err); return -1; }
    // a reference with bins but no pseudo-bin (optional in the spec): the count is unknown (-1)
    int64_t m = 0;
    for (auto& R : bai) {
        auto it = R.bins.find(37450);
        if (it != R.bins.end() && it->second.size() >= 2) m += (int64_t)it->second[1].first;
        else if (!R.bins.empty()) { set_err("BAI without pseudo-bins: mapped count unknown"); return -1; }
    }
    return m;
}

// per region: the compressed bytes its records span in the BAI (the shard plan's weights)
int ccio_bai_region_bytes(const char* path, int32_t n, const int32_t* tid, const int64_t* beg, const int64_t* end,
                          int64_t* out) {
    wait_path(path);
    std::vector<BaiRef> bai;
    std::string err;
    if (!read_bai(std::string(path) + ".bai", bai, err)) { set_err(err); return -1; }
    std::vector<uint32_t> bins;
    for (int32_t i = 0; i < n; ++i) {
        out[i] = 0;
        const int32_t t = tid[i];
        if (t < 0 || t >= (int32_t)bai.size() || end[i] <= beg[i] || bai[t].lin.empty()) continue;
        const int64_t b0 = std::max<int64_t>(beg[i], 0);
        if ((size_t)(b0 >> 14) >= bai[t].lin.size() || bai[t].first == ~0ULL) continue;
        const uint64_t v0 = bai[t].start(b0);
        uint64_t vmax = 0;
        reg2bins(b0, end[i], bins);
        for (uint32_t bn : bins) {
            auto it = bai[t].bins.find(bn);
            if (it == bai[t].bins.end()) continue;
            for (auto& c : it->second)
                if (c.second > v0) vmax = std::max(vmax, c.second);
        }
        if (vmax > v0) out[i] = (int64_t)((vmax >> 16) - (v0 >> 16)) * 4 + (int64_t)((vmax & 0xffff) + 1);
    }
    return 0;
}

// ------------------------------------------------------------------ fastq2bam UMI extraction
// extract_barcodes.py:144-481, the per-pair work (the stats text and the histogram plot stay in
// the Python host, consensuscruncher_amd/extract_barcodes.py).  Both FASTQs are read whole ('gz' in
// the read-1 name: gzip, as :200-205 decide), indexed record by record (Biopython's FASTQ grammar:
// '@' title, sequence lines up to '+', quality lines up to the sequence length; id = the title up to
// the first whitespace), then the pairs are split over threads and each thread formats its pairs
// into its own buffers, which are written in pair order.
namespace {
struct FqRec {
    const char *id, *seq, *qual;
    int32_t idlen, len;
};

bool read_text(const char* path, bool gz, std::string& out) {
    out.clear();
    if (gz) {
        gzFile g = gzopen(path, "rb");
        if (!g) return false;
        char buf[1 << 16];
        int k;
        while ((k = gzread(g, buf, sizeof buf)) > 0) out.append(buf, k);
        const bool ok = k == 0;
        gzclose(g);
        return ok;
    }
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    char buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, k);
    fclose(f);
    return true;
}

// one line [p, eol) without the line break (and a trailing '\r'); returns the next line's start
const char* next_line(const char* p, const char* end, const char** eol) {
    const char* nl = (const char*)memchr(p, '\n', end - p);
    const char* e = nl ? nl : end;
    *eol = (e > p && e[-1] == '\r') ? e - 1 : e;
    return nl ? nl + 1 : end;
}

bool index_fastq(const std::string& t, std::vector<FqRec>& recs, std::string& err) {
    const char* p = t.data();
    const char* end = p + t.size();
    while (p < end) {
        const char* eol;
        const char* nx = next_line(p, end, &eol);
        if (eol == p) { p = nx; continue; }   // blank lines between records
        if (*p != '@') { err = "FASTQ record does not start with '@'"; return false; }
        FqRec r;
        r.id = p + 1;
        const char* q = r.id;
        while (q < eol && *q != ' ' && *q != '\t') ++q;
        r.idlen = (int32_t)(q - r.id);
        p = nx;
        // sequence: one line (multi-line records are rejected rather than silently joined)
        if (p >= end) { err = "FASTQ record truncated"; return false; }
        nx = next_line(p, end, &eol);
        r.seq = p;
        r.len = (int32_t)(eol - p);
        p = nx;
        if (p >= end || *p != '+') { err = "FASTQ record: expected a single sequence line and '+'"; return false; }
        p = next_line(p, end, &eol);
        if (p >= end && r.len > 0) { err = "FASTQ record truncated"; return false; }
        nx = next_line(p, end, &eol);
        if ((int32_t)(eol - p) != r.len) { err = "FASTQ record: quality length differs from sequence length"; return false; }
        r.qual = p;
        p = nx;
        recs.push_back(r);
    }
    return true;
}

inline bool acgt_only(const char* s, int32_t n) {
    for (int32_t i = 0; i < n; ++i)
        if (s[i] != 'A' && s[i] != 'C' && s[i] != 'G' && s[i] != 'T') return false;
    return true;
}

inline int nuc_col(char c) {
    switch (c) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        default: return 4;
    }
}

void put_read(std::string& o, const FqRec& r, const std::string& bc, char mate, int32_t cut) {
    cut = std::min(cut, r.len);   // read[blen:] of a read shorter than the barcode: empty
    o += '@';
    o.append(r.id, r.idlen);
    o += '|';
    o += bc;
    o += '/';
    o += mate;
    o += '\n';
    o.append(r.seq + cut, r.len - cut);
    o += "\n+\n";
    o.append(r.qual + cut, r.len - cut);
    o += '\n';
}
}  // namespace

int ccio_extract_barcodes(const char* read1, const char* read2, const char* out_prefix, const char* pattern,
                          const char* const* blist, int32_t nblist, int nthreads, int64_t* counts,
                          int64_t* r1_hist, int64_t* r2_hist, int64_t* n_written) {
    if (!read1 || !read2 || !out_prefix || !counts || !r1_hist || !r2_hist) { set_err("null argument"); return -1; }
    const bool by_pattern = pattern != nullptr;
    if (!by_pattern && (!blist || nblist <= 0)) { set_err("no barcode pattern or list"); return -1; }
    const bool gz = strstr(read1, "gz") != nullptr;
    std::string t1, t2;
    if (!read_text(read1, gz, t1)) { set_err(std::string("cannot read ") + read1); return -1; }
    if (!read_text(read2, gz, t2)) { set_err(std::string("cannot read ") + read2); return -1; }
    std::vector<FqRec> a, b;
    std::string err;
    if (!index_fastq(t1, a, err) || !index_fastq(t2, b, err)) { set_err(err); return -1; }
    // zip(read1, read2) stops at the shorter file; `assert r1.id == r2.id` (:291) stops at the
    // first pair whose ids differ, after the pairs before it were written
    int64_t n = (int64_t)std::min(a.size(), b.size());
    int rc = 0;
    // pattern: barcode (N) and spacer positions (:237-242); list: the distinct lengths, longest first
    const int32_t plen = by_pattern ? (int32_t)strlen(pattern) : 0;
    std::vector<int32_t> bidx, sidx;
    std::string spacer;
    for (int32_t i = 0; i < plen; ++i) {
        if (pattern[i] == 'N') bidx.push_back(i);
        else { sidx.push_back(i); spacer += pattern[i]; }
    }
    std::unordered_map<std::string, int32_t> lidx;
    std::vector<int32_t> lens;
    int32_t maxlen = plen;
    for (int32_t i = 0; !by_pattern && i < nblist; ++i) {
        const std::string s(blist[i]);
        lidx.emplace(s, i);
        if (std::find(lens.begin(), lens.end(), (int32_t)s.size()) == lens.end()) lens.push_back((int32_t)s.size());
        maxlen = std::max(maxlen, (int32_t)s.size());
    }
    std::sort(lens.rbegin(), lens.rend());
    for (int64_t i = 0; i < n; ++i) {
        if (a[i].idlen != b[i].idlen || memcmp(a[i].id, b[i].id, a[i].idlen) != 0) {
            set_err("read 1 and read 2 ids differ at pair " + std::to_string(i + 1) + " (AssertionError)");
            n = i;
            rc = -2;
            break;
        }
        // pattern mode: a read shorter than the pattern ends the reference in seq_to_mat / indexing;
        // list mode takes read.seq[:blen] as it comes (extract_barcode, :125-138)
        if (by_pattern && (a[i].len < maxlen || b[i].len < maxlen)) {
            set_err("read shorter than the barcode at pair " + std::to_string(i + 1));
            n = i;
            rc = -3;
            break;
        }
    }
    const int nh = by_pattern ? plen * 5 : nblist;
    const int T = std::max(1, std::min<int>(hw_threads(nthreads), (int)std::max<int64_t>(1, n / 4096)));
    struct Part {
        std::string o1, o2, bad1, bad2;
        int64_t spacer = 0, badbc = 0, good = 0;
        std::vector<int64_t> h1, h2;
    };
    std::vector<Part> parts(T);
    parallel_for(n, T, [&](int64_t lo, int64_t hi, int tix) {
        Part& P = parts[tix];
        P.h1.assign(nh, 0);
        P.h2.assign(nh, 0);
        std::string bc;
        for (int64_t i = lo; i < hi; ++i) {
            const FqRec &x = a[i], &y = b[i];
            if (by_pattern) {
                if (!acgt_only(x.seq, plen) || !acgt_only(y.seq, plen)) { ++P.badbc; continue; }
                for (int32_t k = 0; k < plen; ++k) {
                    ++P.h1[5 * k + nuc_col(x.seq[k])];
                    ++P.h2[5 * k + nuc_col(y.seq[k])];
                }
                bool sp = true;
                for (size_t k = 0; k < sidx.size(); ++k)
                    sp = sp && x.seq[sidx[k]] == spacer[k] && y.seq[sidx[k]] == spacer[k];
                if (!sp) { ++P.spacer; continue; }
                ++P.good;
                bc.clear();
                for (int32_t k : bidx) bc += x.seq[k];
                bc += '.';
                for (int32_t k : bidx) bc += y.seq[k];
                put_read(P.o1, x, bc, '1', plen);
                put_read(P.o2, y, bc, '2', plen);
            } else {
                // every length, longest first; a later (shorter) match replaces an earlier one (:347-376).
                // A read shorter than the length gives its whole sequence as the barcode (read.seq[:blen]);
                // such a barcode can only match an entry of its own length, which a later iteration meets.
                int32_t l1 = -1, l2 = -1, e1 = -1, e2 = -1;
                int32_t last1 = 0, last2 = 0;
                for (int32_t bl : lens) {
                    const int32_t k1 = std::min(bl, x.len), k2 = std::min(bl, y.len);
                    last1 = k1;
                    last2 = k2;
                    const bool ok1 = acgt_only(x.seq, k1), ok2 = acgt_only(y.seq, k2);
                    if (!ok1 || !ok2) {
                        ++P.badbc;
                        if (!ok1) { P.bad1.append(x.seq, k1); P.bad1 += '\n'; }
                        if (!ok2) { P.bad2.append(y.seq, k2); P.bad2 += '\n'; }
                        continue;
                    }
                    auto f1 = lidx.find(std::string(x.seq, k1));
                    if (f1 != lidx.end()) { l1 = bl; e1 = f1->second; }
                    auto f2 = lidx.find(std::string(y.seq, k2));
                    if (f2 != lidx.end()) { l2 = bl; e2 = f2->second; }
                }
                if (l1 > 0 && l2 > 0) {
                    ++P.good;
                    ++P.h1[e1];
                    ++P.h2[e2];
                    bc.assign(x.seq, l1 - 1);   // the barcode without its T (:370,376)
                    bc += '.';
                    bc.append(y.seq, l2 - 1);
                    put_read(P.o1, x, bc, '1', l1);
                    put_read(P.o2, y, bc, '2', l2);
                } else {
                    // the barcodes of the last (shortest) length go to the bad-barcode lists (:398-405)
                    ++P.badbc;
                    if (l1 <= 0) { P.bad1.append(x.seq, last1); P.bad1 += '\n'; }
                    if (l2 <= 0) { P.bad2.append(y.seq, last2); P.bad2 += '\n'; }
                }
            }
        }
    });
    const std::string pre(out_prefix);
    auto write_all = [&](const std::string& path, std::string Part::*m) {
        FILE* f = fopen(path.c_str(), "wb");
        if (!f) return false;
        bool ok = true;
        for (Part& P : parts) ok = ok && fwrite((P.*m).data(), 1, (P.*m).size(), f) == (P.*m).size();
        return fclose(f) == 0 && ok;
    };
    if (!write_all(pre + "_barcode_R1.fastq", &Part::o1) || !write_all(pre + "_barcode_R2.fastq", &Part::o2) ||
        (!by_pattern && (!write_all(pre + "_r1_bad_barcodes.txt", &Part::bad1) ||
                         !write_all(pre + "_r2_bad_barcodes.txt", &Part::bad2)))) {
        set_err("cannot write the outputs under " + pre);
        return -1;
    }
    counts[0] = n + (rc ? 1 : 0);   // readpair_count includes the pair the assertion stopped at
    counts[1] = counts[2] = counts[3] = 0;
    for (int k = 0; k < nh; ++k) r1_hist[k] = r2_hist[k] = 0;
    for (Part& P : parts) {
        counts[1] += P.spacer;
        counts[2] += P.badbc;
        counts[3] += P.good;
        for (int k = 0; k < nh && !P.h1.empty(); ++k) { r1_hist[k] += P.h1[k]; r2_hist[k] += P.h2[k]; }
    }
    if (n_written) *n_written = n;
    return rc;
}

// The same extraction with the per-pair decisions made elsewhere (the GPU: cc_extract_barcodes).
// ccio_fq_open reads and indexes both FASTQs and stops where the reference stops (ids differing:
// AssertionError; pattern mode, a read shorter than min_len); ccio_fq_heads hands out the first
// `width` bases of every pair's reads; ccio_fq_write formats the outputs from the decisions: status
// 0 = passing (header barcode bc[i], reads cut by cut1 / cut2), else not written; list mode's
// bad-barcode lines from the per-read masks (bit j: the prefix of length min(lens[j], read length),
// in lens order; bit 31: the prefix of the last length once more).
struct ccio_fq {
    std::string t1, t2;
    std::vector<FqRec> a, b;
    int64_t n = 0;
    int32_t stop = 0;
};

ccio_fq* ccio_fq_open(const char* read1, const char* read2, int32_t min_len, int nthreads) {
    (void)nthreads;
    if (!read1 || !read2) { set_err("null argument"); return nullptr; }
    std::unique_ptr<ccio_fq> f(new ccio_fq());
    const bool gz = strstr(read1, "gz") != nullptr;
    if (!read_text(read1, gz, f->t1)) { set_err(std::string("cannot read ") + read1); return nullptr; }
    if (!read_text(read2, gz, f->t2)) { set_err(std::string("cannot read ") + read2); return nullptr; }
    std::string err;
    if (!index_fastq(f->t1, f->a, err) || !index_fastq(f->t2, f->b, err)) { set_err(err); return nullptr; }
    int64_t n = (int64_t)std::min(f->a.size(), f->b.size());
    for (int64_t i = 0; i < n; ++i) {
        const FqRec &x = f->a[i], &y = f->b[i];
        if (x.idlen != y.idlen || memcmp(x.id, y.id, x.idlen) != 0) {
            set_err("read 1 and read 2 ids differ at pair " + std::to_string(i + 1) + " (AssertionError)");
            n = i;
            f->stop = -2;
            break;
        }
        if (x.len < min_len || y.len < min_len) {
            set_err("read shorter than the barcode at pair " + std::to_string(i + 1));
            n = i;
            f->stop = -3;
            break;
        }
    }
    f->n = n;
    return f.release();
}

void ccio_fq_close(ccio_fq* f) { delete f; }

int ccio_fq_info(ccio_fq* f, int64_t* n, int32_t* stop) {
    if (!f || !n || !stop) return -1;
    *n = f->n;
    *stop = f->stop;
    return 0;
}

int ccio_fq_heads(ccio_fq* f, int32_t width, uint8_t* h1, uint8_t* h2, int32_t* len1, int32_t* len2) {
    if (!f || width <= 0 || (f->n > 0 && (!h1 || !h2 || !len1 || !len2))) { set_err("bad arguments"); return -1; }
    parallel_chunks(f->n, hw_threads(0), 65536, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) {
            const FqRec &x = f->a[i], &y = f->b[i];
            uint8_t* p = h1 + i * (int64_t)width;
            uint8_t* q = h2 + i * (int64_t)width;
            memset(p, 0, width);
            memset(q, 0, width);
            memcpy(p, x.seq, std::min(x.len, width));
            memcpy(q, y.seq, std::min(y.len, width));
            len1[i] = x.len;
            len2[i] = y.len;
        }
    });
    return 0;
}

int ccio_fq_write(ccio_fq* f, const char* out_prefix, int list_mode, const uint8_t* status, const char* bc,
                  int32_t bc_stride, const int32_t* cut1, const int32_t* cut2, const uint32_t* bad1,
                  const uint32_t* bad2, const int32_t* lens, int32_t nlens, int nthreads) {
    if (!f || !out_prefix || (f->n > 0 && (!status || !bc || !cut1 || !cut2)) ||
        (list_mode && f->n > 0 && (!bad1 || !bad2 || !lens || nlens <= 0))) { set_err("bad arguments"); return -1; }
    const int64_t n = f->n;
    const int T = std::max(1, std::min<int>(hw_threads(nthreads), (int)std::max<int64_t>(1, n / 4096)));
    struct Part {
        std::string o1, o2, bad1, bad2;
    };
    std::vector<Part> parts(T);
    auto bad_lines = [&](std::string& o, const FqRec& r, uint32_t m) {
        for (int32_t j = 0; j < nlens; ++j)
            if (m & (1u << j)) { o.append(r.seq, std::min(lens[j], r.len)); o += '\n'; }
        if (m & (1u << 31)) { o.append(r.seq, std::min(lens[nlens - 1], r.len)); o += '\n'; }
    };
    parallel_for(n, T, [&](int64_t lo, int64_t hi, int tix) {
        Part& P = parts[tix];
        std::string b;
        for (int64_t i = lo; i < hi; ++i) {
            const FqRec &x = f->a[i], &y = f->b[i];
            if (list_mode) {
                bad_lines(P.bad1, x, bad1[i]);
                bad_lines(P.bad2, y, bad2[i]);
            }
            if (status[i] != 0) continue;
            b.assign(bc + i * (int64_t)bc_stride, strnlen(bc + i * (int64_t)bc_stride, (size_t)bc_stride));
            put_read(P.o1, x, b, '1', cut1[i]);
            put_read(P.o2, y, b, '2', cut2[i]);
        }
    });
    const std::string pre(out_prefix);
    auto write_all = [&](const std::string& path, std::string Part::*m) {
        FILE* fp = fopen(path.c_str(), "wb");
        if (!fp) return false;
        bool ok = true;
        for (Part& P : parts) ok = ok && fwrite((P.*m).data(), 1, (P.*m).size(), fp) == (P.*m).size();
        return fclose(fp) == 0 && ok;
    };
    if (!write_all(pre + "_barcode_R1.fastq", &Part::o1) || !write_all(pre + "_barcode_R2.fastq", &Part::o2) ||
        (list_mode && (!write_all(pre + "_r1_bad_barcodes.txt", &Part::bad1) ||
                       !write_all(pre + "_r2_bad_barcodes.txt", &Part::bad2)))) {
        set_err("cannot write the outputs under " + pre);
        return -1;
    }
    return 0;
}

// Columnar writer used by the synthetic generator (consensuscruncher_amd/synth.py).
int ccio_write_columns(const char* path, const char* header_text, int32_t nref, const char* const* ref_names,
                       const int32_t* ref_lens, int64_t n, const int32_t* tid, const int32_t* pos,
                       const int32_t* mtid, const int32_t* mpos, const int32_t* tlen, const uint16_t* flag,
                       const uint8_t* mapq, const uint8_t* qn_blob, const int64_t* qn_off, const int32_t* cig_id,
                       const uint32_t* cig_ops, const int64_t* cig_off, int32_t read_len, const uint8_t* seq_ascii,
                       const uint8_t* qual, const int32_t* rg_id, const char* const* rg_vals, int level,
                       int nthreads) {
    std::string hdr = "BAM\1";
    std::string ht(header_text);
    wr32(hdr, (int32_t)ht.size());
    hdr += ht;
    wr32(hdr, nref);
    for (int i = 0; i < nref; ++i) {
        std::string nm(ref_names[i]);
        wr32(hdr, (int32_t)nm.size() + 1);
        hdr += nm;
        hdr.push_back('\0');
        wr32(hdr, ref_lens[i]);
    }
    static const int8_t code[256] = {
#define X15 15,15,15,15,15,15,15,15,15,15,15,15,15,15,15,15
        X15, X15, X15, X15,
        15, 1, 15, 2, 15, 15, 15, 4, 15, 15, 15, 15, 15, 15, 15, 15,   // '@'..'O': A=1 C=2 G=4 N=15
        15, 15, 15, 15, 8, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15, 15,  // 'P'..'_': T=8
        X15, X15, X15, X15, X15, X15, X15, X15, X15, X15
#undef X15
    };
    int T = hw_threads(nthreads);
    std::vector<std::string> parts(T);
    parallel_for(n, T, [&](int64_t s, int64_t e, int t) {
        std::string& out = parts[t];
        for (int64_t i = s; i < e; ++i) {
            std::string body;
            int64_t ql = qn_off[i + 1] - qn_off[i];
            int c = cig_id[i];
            int64_t nc = c >= 0 ? cig_off[c + 1] - cig_off[c] : 0;
            int64_t rlen = 0;
            for (int64_t k = 0; k < nc; ++k) {
                uint32_t v = cig_ops[cig_off[c] + k];
                uint32_t op = v & 0xf;
                if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rlen += v >> 4;
            }
            bool unm = flag[i] & 4;
            int64_t p = pos[i];
            int64_t endp = p + ((!unm && rlen) ? rlen : 1);
            wr32(body, tid[i]);
            wr32(body, pos[i]);
            body.push_back((char)(ql + 1));
            body.push_back((char)mapq[i]);
            wru16(body, (uint16_t)reg2bin(p < 0 ? 0 : p, p < 0 ? 1 : endp));
            wru16(body, (uint16_t)nc);
            wru16(body, flag[i]);
            wr32(body, read_len);
            wr32(body, mtid[i]);
            wr32(body, mpos[i]);
            wr32(body, tlen[i]);
            body.append((const char*)qn_blob + qn_off[i], ql);
            body.push_back('\0');
            for (int64_t k = 0; k < nc; ++k) body.append((const char*)&cig_ops[cig_off[c] + k], 4);
            const uint8_t* sq = seq_ascii + (size_t)i * read_len;
            for (int32_t k = 0; k < read_len; k += 2) {
                uint8_t hi = code[sq[k]], lo = (k + 1 < read_len) ? code[sq[k + 1]] : 0;
                body.push_back((char)((hi << 4) | lo));
            }
            body.append((const char*)qual + (size_t)i * read_len, read_len);
            if (rg_id && rg_id[i] >= 0) {
                body += "RGZ";
                body += rg_vals[rg_id[i]];
                body.push_back('\0');
            }
            wr32(out, (int32_t)body.size());
            out += body;
        }
    });
    FILE* f = fopen(path, "wb");
    if (!f) { set_err(std::string("cannot write ") + path); return -1; }
    std::string all = hdr;
    for (auto& p : parts) { all += p; std::string().swap(p); }
    bool ok = bgzf_deflate_write(f, (const uint8_t*)all.data(), all.size(), level, T);
    fclose(f);
    return ok ? 0 : -1;
}

}  // extern "C"
