// cc_oracle.cpp — a second CPU restatement of ConsensusCruncher's consensus mode, in C++.
//
// TEST INFRASTRUCTURE ONLY.  Loaded (oracle/cc_oracle_native.py, ctypes) by tests/, by
// __graft_entry__.smoke() and by the cpu_baseline leg of bench.py -- never by the product, which
// fails loudly when its HIP library is missing.  It is the same dictionary program as
// oracle/cc_oracle.py (the pinned Python restatement), written for speed so that parity can be
// checked at sizes the Python oracle cannot reach and so that the CPU baseline is a compiled,
// consensus-only time.  Pinning: tests/test_oracle_native.py requires it to reproduce every case of
// tests/golden (outputs of the unmodified reference, oracle/make_golden.py) record for record, and
// to agree with oracle/cc_oracle.py on seeded samples.
//
// Reference semantics restated here (file:line):
//   which_read / which_strand / cigar_order     consensus_helper.py:57-196
//   sscs_qname / unique_tag                      consensus_helper.py:199-305
//   read_bam (filters, pair_dict, dictionaries)  consensus_helper.py:308-506
//   read_mode / consensus_flag / create_aligned_segment   consensus_helper.py:509-619
//   duplex_tag                                   consensus_helper.py:639-683
//   bed_separator                                consensus_helper.py:38-54
//   consensus_maker                              SSCS_maker.py:81-168
//   SSCS main (region loop, stats, families)     SSCS_maker.py:183-425
//   dcs_consensus_tag / duplex_consensus / main  DCS_maker.py:60-123, 130-317
//   duplex_consensus (Q>29) / main               singleton_correction.py:61-86, 118-345
//   samtools sort / merge stand-in               oracle/samtools_shim.py (stable, file-order ties)
// Mode ties pick the first-seen value (the fixtures patch randint to its lower bound).
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <exception>
#include <thread>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

thread_local std::string g_err;

struct OracleError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------ BGZF / BAM codec
std::string read_file(const std::string& path) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) throw OracleError("cannot open " + path);
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::string s((size_t)std::max(n, 0L), '\0');
    const size_t got = n > 0 ? fread(&s[0], 1, (size_t)n, f) : 0;
    fclose(f);
    if ((long)got != n) throw OracleError("short read " + path);
    return s;
}

// Runs fn(i) for i in [0, n) over the host's threads (the I/O of the oracle only: blocks and
// records are independent; the consensus program itself stays single-threaded).
template <typename F>
void parallel_for(size_t n, F fn) {
    size_t nt = std::min<size_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
    if (const char* e = getenv("CC_ORACLE_THREADS")) nt = std::max(1, atoi(e));
    nt = std::min(nt, std::max<size_t>(n / 64, 1));
    if (nt <= 1) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    std::atomic<size_t> next(0);
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(nt);
    for (size_t t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            try {
                for (size_t i; (i = next.fetch_add(64)) < n;)
                    for (size_t k = i; k < std::min(n, i + 64); ++k) fn(k);
            } catch (...) {
                err[t] = std::current_exception();
            }
        });
    for (auto& x : th) x.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}

std::string bgzf_inflate(const std::string& in) {
    struct Blk { size_t cdata_off, clen, out_off; uint32_t isize; };
    std::vector<Blk> blks;
    size_t off = 0, total = 0;
    while (off + 18 <= in.size()) {
        const uint8_t* h = (const uint8_t*)in.data() + off;
        if (h[0] != 31 || h[1] != 139) throw OracleError("not a BGZF file");
        const uint16_t xlen = (uint16_t)(h[10] | (h[11] << 8));
        int bsize = -1;
        for (size_t x = 12; x + 4 <= 12u + xlen;) {
            const uint16_t slen = (uint16_t)(h[x + 2] | (h[x + 3] << 8));
            if (h[x] == 'B' && h[x + 1] == 'C' && slen == 2) bsize = h[x + 4] | (h[x + 5] << 8);
            x += 4 + slen;
        }
        if (bsize < 0) throw OracleError("BGZF block without BC field");
        if (off + (size_t)bsize + 1 > in.size()) throw OracleError("truncated BGZF block");
        const size_t cdata = (size_t)bsize - xlen - 19;
        const uint8_t* c = h + 12 + xlen;
        const uint32_t isize = (uint32_t)c[cdata + 4] | ((uint32_t)c[cdata + 5] << 8) | ((uint32_t)c[cdata + 6] << 16) |
                               ((uint32_t)c[cdata + 7] << 24);
        blks.push_back({off + 12 + xlen, cdata, total, isize});
        total += isize;
        off += (size_t)bsize + 1;
    }
    std::string out(total, '\0');
    parallel_for(blks.size(), [&](size_t i) {
        const Blk& b = blks[i];
        if (!b.isize) return;
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        inflateInit2(&zs, -15);
        zs.next_in = (Bytef*)in.data() + b.cdata_off;
        zs.avail_in = (uInt)b.clen;
        zs.next_out = (Bytef*)&out[b.out_off];
        zs.avail_out = b.isize;
        const int rc = inflate(&zs, Z_FINISH);
        inflateEnd(&zs);
        if (rc != Z_STREAM_END) throw OracleError("BGZF inflate failed");
    });
    return out;
}

void put_le(std::string& s, uint64_t v, int n) {
    for (int i = 0; i < n; ++i) s.push_back((char)((v >> (8 * i)) & 0xff));
}

std::string bgzf_deflate(const std::string& data) {
    const size_t B = 65280, nb = (data.size() + B - 1) / B;
    std::vector<std::string> parts(nb + 1);
    auto block = [&](const char* p, size_t n, std::string& out) {
        std::vector<uint8_t> buf(compressBound((uLong)n) + 64);
        z_stream zs;
        memset(&zs, 0, sizeof(zs));
        deflateInit2(&zs, 1, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
        zs.next_in = (Bytef*)p;
        zs.avail_in = (uInt)n;
        zs.next_out = buf.data();
        zs.avail_out = (uInt)buf.size();
        deflate(&zs, Z_FINISH);
        const size_t clen = zs.total_out;
        deflateEnd(&zs);
        const uint32_t crc = (uint32_t)crc32(0, (const Bytef*)p, (uInt)n);
        const size_t bsize = clen + 25;   // BSIZE = total block size - 1 (18-B header, 8-B trailer)
        const uint8_t hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 'B', 'C', 2, 0,
                                 (uint8_t)(bsize & 0xff), (uint8_t)(bsize >> 8)};
        out.append((const char*)hdr, 18);
        out.append((const char*)buf.data(), clen);
        put_le(out, crc, 4);
        put_le(out, n, 4);
    };
    parallel_for(nb, [&](size_t i) { block(data.data() + i * B, std::min(B, data.size() - i * B), parts[i]); });
    block(nullptr, 0, parts[nb]);   // EOF marker
    size_t tot = 0;
    for (auto& s : parts) tot += s.size();
    std::string out;
    out.reserve(tot);
    for (auto& s : parts) out += s;
    return out;
}

int32_t rd32(const char* p) { int32_t v; memcpy(&v, p, 4); return v; }
uint32_t rdu32(const char* p) { uint32_t v; memcpy(&v, p, 4); return v; }
uint16_t rd16(const char* p) { uint16_t v; memcpy(&v, p, 2); return v; }

const char* SEQ_NT16 = "=ACMGRSVTWYHKDBN";
const char* CIGAR_OPS = "MIDNSHP=XB";

struct Header {
    std::string raw;                     // magic .. refs, written back unchanged (template=)
    std::vector<std::string> refs;
    int32_t tid(const std::string& name) const {
        for (size_t i = 0; i < refs.size(); ++i)
            if (refs[i] == name) return (int32_t)i;
        return -1;
    }
};

struct Rec {
    std::string qname;
    uint16_t flag = 0;
    int32_t tid = -1, pos = -1, mtid = -1, mpos = -1, tlen = 0;
    uint8_t mapq = 0;
    uint16_t bin = 0;
    std::vector<uint32_t> cigar;
    std::string seq;        // ASCII (SEQ_NT16), empty: '*'
    std::string qual;       // raw phred bytes; empty with qual_missing or no seq
    bool qual_missing = true;
    std::string aux;        // raw aux bytes
    std::string raw;        // the record as read (bin zeroed): record equality, pysam __eq__
    uint64_t content = 0;   // digest (tests)
    bool is_reverse() const { return flag & 0x10; }
    bool is_unmapped() const { return flag & 0x4; }
    std::string cigarstring() const {
        std::string s;
        for (uint32_t c : cigar) s += std::to_string(c >> 4) + CIGAR_OPS[c & 0xf];
        return s.empty() ? "None" : s;   // str(None) in the reference's tag strings
    }
    int infer_query_length() const {   // -1: None (no cigar)
        if (cigar.empty()) return -1;
        int n = 0;
        for (uint32_t c : cigar) {
            const uint32_t op = c & 0xf;
            if (op == 0 || op == 1 || op == 4 || op == 7 || op == 8) n += (int)(c >> 4);
        }
        return n;
    }
    int32_t endpos() const {
        int32_t rl = 0;
        if (!(flag & 4))
            for (uint32_t c : cigar) {
                const uint32_t op = c & 0xf;
                if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += (int32_t)(c >> 4);
            }
        return pos + (rl ? rl : 1);
    }
    bool get_rg(std::string& v, char& ty) const {
        size_t p = 0;
        while (p + 3 <= aux.size()) {
            const char t0 = aux[p], t1 = aux[p + 1], typ = aux[p + 2];
            size_t q = p + 3, vlen = 0;
            switch (typ) {
                case 'A': case 'c': case 'C': vlen = 1; break;
                case 's': case 'S': vlen = 2; break;
                case 'i': case 'I': case 'f': vlen = 4; break;
                case 'Z': case 'H': vlen = aux.find('\0', q) - q + 1; break;
                case 'B': {
                    const char sub = aux[q];
                    const uint32_t cnt = rdu32(aux.data() + q + 1);
                    const size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
                    vlen = 5 + cnt * es;
                    break;
                }
                default: throw OracleError("bad aux type");
            }
            if (t0 == 'R' && t1 == 'G') {
                ty = typ;
                if (typ == 'Z') v = aux.substr(q, vlen - 1);
                else if (typ == 'A') v = aux.substr(q, 1);
                else throw OracleError("RG tag of a non-string type");
                return true;
            }
            p = q + vlen;
        }
        return false;
    }
};

uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ULL; }
    return h;
}

void hash_content(Rec& r) {
    uint64_t h = 0xcbf29ce484222325ULL;
    h = fnv(h, r.qname.data(), r.qname.size());
    h = fnv(h, &r.flag, 2); h = fnv(h, &r.tid, 4); h = fnv(h, &r.pos, 4); h = fnv(h, &r.mapq, 1);
    h = fnv(h, r.cigar.data(), 4 * r.cigar.size()); h = fnv(h, &r.mtid, 4); h = fnv(h, &r.mpos, 4);
    h = fnv(h, &r.tlen, 4); h = fnv(h, r.seq.data(), r.seq.size());
    const uint8_t qm = r.qual_missing; h = fnv(h, &qm, 1); h = fnv(h, r.qual.data(), r.qual.size());
    h = fnv(h, r.aux.data(), r.aux.size());
    r.content = h;
}

// pysam's AlignedSegment __eq__ for records read from a file: every field, i.e. the record bytes
bool same_content(const Rec& a, const Rec& b) { return a.raw == b.raw; }

struct Bam {
    Header h;
    std::vector<Rec> recs;
    int sorted = -1;   // (tid, pos) order, computed on the first region fetch
};

Bam read_bam(const std::string& path) {
    const std::string buf = bgzf_inflate(read_file(path));
    Bam b;
    if (buf.size() < 12 || memcmp(buf.data(), "BAM\1", 4)) throw OracleError("not a BAM file: " + path);
    size_t p = 4;
    const int32_t ltext = rd32(buf.data() + p);
    p += 4 + ltext;
    const int32_t nref = rd32(buf.data() + p);
    p += 4;
    for (int32_t i = 0; i < nref; ++i) {
        const int32_t ln = rd32(buf.data() + p);
        b.h.refs.emplace_back(buf.data() + p + 4, ln - 1);
        p += 4 + ln + 4;
    }
    b.h.raw = buf.substr(0, p);
    std::vector<size_t> offs;
    while (p + 4 <= buf.size()) {
        const int32_t bs = rd32(buf.data() + p);
        if (bs < 32 || p + 4 + (size_t)bs > buf.size()) throw OracleError("truncated BAM record: " + path);
        offs.push_back(p);
        p += 4 + (size_t)bs;
    }
    b.recs.resize(offs.size());
    parallel_for(offs.size(), [&](size_t i) {
        const int32_t bs = rd32(buf.data() + offs[i]);
        const char* d = buf.data() + offs[i] + 4;
        Rec& r = b.recs[i];
        r.tid = rd32(d); r.pos = rd32(d + 4);
        const uint8_t lqn = (uint8_t)d[8];
        r.mapq = (uint8_t)d[9];
        r.bin = rd16(d + 10);
        const uint16_t ncig = rd16(d + 12);
        r.flag = rd16(d + 14);
        const int32_t lseq = rd32(d + 16);
        r.mtid = rd32(d + 20); r.mpos = rd32(d + 24); r.tlen = rd32(d + 28);
        const char* q = d + 32;
        r.qname.assign(q, lqn - 1);
        q += lqn;
        r.cigar.resize(ncig);
        for (uint16_t k = 0; k < ncig; ++k) r.cigar[k] = rdu32(q + 4 * k);
        q += 4 * ncig;
        r.seq.resize(lseq);
        for (int32_t i2 = 0; i2 < lseq; ++i2) r.seq[i2] = SEQ_NT16[((uint8_t)q[i2 >> 1] >> (4 * (1 - (i2 & 1)))) & 0xf];
        q += (lseq + 1) / 2;
        r.qual_missing = lseq == 0 || (uint8_t)q[0] == 0xff;
        if (!r.qual_missing) r.qual.assign(q, lseq);
        q += lseq;
        r.aux.assign(q, d + bs - q);
        r.raw.assign(d, bs);
        r.raw[10] = r.raw[11] = 0;
    });
    return b;
}

int reg2bin(int beg, int end) {
    --end;
    if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
    if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
    if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
    if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
    if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
    return 0;
}

int nt16_code(char c) {
    const char u = (char)toupper((unsigned char)c);
    const char* p = strchr(SEQ_NT16, u);
    return (p && u) ? (int)(p - SEQ_NT16) : 15;
}

void encode(const Rec& r, std::string& out) {
    std::string b;
    put_le(b, (uint32_t)r.tid, 4);
    put_le(b, (uint32_t)r.pos, 4);
    const std::string qn = r.qname.empty() ? "*" : r.qname;
    b.push_back((char)(qn.size() + 1));
    b.push_back((char)r.mapq);
    put_le(b, r.bin, 2);
    put_le(b, r.cigar.size(), 2);
    put_le(b, r.flag, 2);
    put_le(b, r.seq.size(), 4);
    put_le(b, (uint32_t)r.mtid, 4);
    put_le(b, (uint32_t)r.mpos, 4);
    put_le(b, (uint32_t)r.tlen, 4);
    b += qn;
    b.push_back('\0');
    for (uint32_t c : r.cigar) put_le(b, c, 4);
    const size_t ls = r.seq.size();
    std::string sb((ls + 1) / 2, '\0');
    for (size_t i = 0; i < ls; ++i) {
        const int code = nt16_code(r.seq[i]);
        if (i & 1) sb[i >> 1] = (char)(sb[i >> 1] | code);
        else sb[i >> 1] = (char)(code << 4);
    }
    b += sb;
    if (r.qual_missing) b += std::string(ls, (char)0xff);
    else b += r.qual;
    b += r.aux;
    put_le(out, b.size(), 4);
    out += b;
}

void write_bam(const std::string& path, const Header& h, const std::vector<Rec>& recs) {
    const size_t C = 4096, nc = (recs.size() + C - 1) / C;
    std::vector<std::string> chunk(nc);
    parallel_for(nc, [&](size_t i) {
        for (size_t k = i * C; k < std::min(recs.size(), (i + 1) * C); ++k) encode(recs[k], chunk[i]);
    });
    std::string data = h.raw;
    for (auto& s : chunk) data += s;
    const std::string z = bgzf_deflate(data);
    std::ofstream f(path, std::ios::binary);
    if (!f) throw OracleError("cannot write " + path);
    f.write(z.data(), (std::streamsize)z.size());
}

// ------------------------------------------------------------------ keys (consensus_helper.py:57-305)
int read_number(int f) {   // 1 R1, 2 R2, 0 None
    switch (f) {
        case 99: case 83: case 67: case 115: case 81: case 97: case 65: case 113: return 1;
        case 147: case 163: case 131: case 179: case 161: case 145: case 129: case 177: return 2;
        default: return 0;
    }
}
const char* read_number_str(int f) {
    const int n = read_number(f);
    return n == 1 ? "R1" : n == 2 ? "R2" : "None";
}
// 1 pos, 2 neg, 0 None
int strand_of(const Rec& r) {
    switch (r.flag) {
        case 99: case 147: case 67: case 131: return 1;
        case 83: case 163: case 115: case 179: return 2;
        case 65: case 129: case 113: case 177: case 81: case 161: case 97: case 145: {
            const int num = read_number(r.flag);
            const int32_t a = r.tid, b = r.mtid, x = r.pos, y = r.mpos;
            if (num == 1) return (a < b || (a == b && x < y)) ? 1 : 2;
            return (a > b || (a == b && x > y)) ? 1 : 2;
        }
        default: return 0;
    }
}
const char* strand_str(int s) { return s == 1 ? "pos" : s == 2 ? "neg" : "None"; }

std::string ordered_cigars(const Rec& first, const Rec& second) {
    const int s = strand_of(first), num = read_number(first.flag);
    const bool own_first = (s == 1 && num == 1) || (s == 2 && num == 2);
    const Rec& a = own_first ? first : second;
    const Rec& b = own_first ? second : first;
    return a.cigarstring() + "_" + b.cigarstring();
}

std::string molecule_name(const Rec& first, const Rec& second, const std::string& bc, const std::string& cig) {
    int32_t c1 = first.tid, p1 = first.pos, c2 = second.tid, p2 = second.pos;
    if (c1 > c2 || (c1 == c2 && p1 > p2)) { std::swap(c1, c2); std::swap(p1, p2); }
    const int64_t tl = first.tlen < 0 ? -(int64_t)first.tlen : first.tlen;
    return bc + "_" + std::to_string(c1) + "_" + std::to_string(p1) + "_" + std::to_string(c2) + "_" +
           std::to_string(p2) + "_" + cig + "_" + strand_str(strand_of(first)) + "_" + std::to_string(tl);
}

std::string read_end_key(const Rec& r, const std::string& bc, const std::string& cig) {
    return bc + "_" + std::to_string(r.tid) + "_" + std::to_string(r.pos) + "_" + std::to_string(r.mtid) + "_" +
           std::to_string(r.mpos) + "_" + cig + "_" + (r.is_reverse() ? "rev" : "fwd") + "_" + read_number_str(r.flag);
}

std::vector<std::string> split(const std::string& s, const std::string& sep) {
    std::vector<std::string> out;
    size_t p = 0;
    while (true) {
        const size_t q = s.find(sep, p);
        if (q == std::string::npos) { out.push_back(s.substr(p)); return out; }
        out.push_back(s.substr(p, q - p));
        p = q + sep.size();
    }
}

std::string complement_key(const std::string& key) {
    std::vector<std::string> parts = split(key, "_");
    std::string& bc = parts[0];
    const size_t k = bc.find('.');
    if (k != std::string::npos) bc = bc.substr(k + 1) + "." + bc.substr(0, k);
    else { const size_t h = bc.size() / 2; bc = bc.substr(h) + bc.substr(0, h); }
    if (parts.size() <= 8) throw OracleError("IndexError: duplex_tag of a short tag");
    parts[8] = parts[8] == "R1" ? "R2" : "R1";
    std::string out = parts[0];
    for (size_t i = 1; i < parts.size(); ++i) out += "_" + parts[i];
    return out;
}

// ------------------------------------------------------------------ insertion-ordered dictionaries
template <typename V>
struct OrderedMap {   // Python dict semantics: insertion order, deletion, re-insertion at the end
    std::unordered_map<std::string, size_t> idx;
    std::vector<std::pair<std::string, V>> items;
    std::vector<uint8_t> live;
    size_t n_live = 0;
    bool frozen = false;   // no compaction while the entries are walked
    V* find(const std::string& k) {
        auto it = idx.find(k);
        return it == idx.end() ? nullptr : &items[it->second].second;
    }
    bool has(const std::string& k) const { return idx.count(k) != 0; }
    V& insert(const std::string& k, V v) {
        idx[k] = items.size();
        items.emplace_back(k, std::move(v));
        live.push_back(1);
        ++n_live;
        return items.back().second;
    }
    V& get_or_insert(const std::string& k) {
        V* p = find(k);
        return p ? *p : insert(k, V());
    }
    void erase(const std::string& k) {
        auto it = idx.find(k);
        if (it == idx.end()) throw OracleError("KeyError: " + k);
        live[it->second] = 0;
        items[it->second].second = V();
        idx.erase(it);
        --n_live;
        if (!frozen && items.size() > 64 && n_live * 4 < items.size()) compact();
    }
    void compact() {
        std::vector<std::pair<std::string, V>> ni;
        std::vector<uint8_t> nl;
        ni.reserve(n_live);
        for (size_t i = 0; i < items.size(); ++i)
            if (live[i]) { idx[items[i].first] = ni.size(); ni.push_back(std::move(items[i])); nl.push_back(1); }
        items.swap(ni);
        live.swap(nl);
    }
    // for key in list(d): the keys live now, in order; fn may delete entries (not insert)
    template <typename F>
    void walk(F fn) {
        frozen = true;
        const size_t n = items.size();
        for (size_t i = 0; i < n; ++i)
            if (live[i]) fn(items[i].first);
        frozen = false;
        if (items.size() > 64 && n_live * 4 < items.size()) compact();
    }
    std::vector<std::string> keys() const {   // list(d): a snapshot in order
        std::vector<std::string> k;
        k.reserve(n_live);
        for (size_t i = 0; i < items.size(); ++i)
            if (live[i]) k.push_back(items[i].first);
        return k;
    }
    void clear() { idx.clear(); items.clear(); live.clear(); n_live = 0; }
};

// ------------------------------------------------------------------ read_bam (consensus_helper.py:308-506)
struct Region {
    std::string key, chrom;
    int64_t start = 0, end = 0;
    bool whole = false;
};

std::vector<Region> regions_of(const char* bedfile) {
    std::vector<Region> out;
    if (!bedfile || !*bedfile) {
        Region r;
        r.whole = true;
        out.push_back(r);
        return out;
    }
    std::ifstream f(bedfile);
    if (!f) throw OracleError(std::string("cannot open bed file ") + bedfile);
    OrderedMap<std::pair<int64_t, int64_t>> table;   // OrderedDict: a repeated key keeps its place
    std::string line;
    while (std::getline(f, line)) {
        const std::vector<std::string> col = split(line, "\t");
        if (col.size() < 4) throw OracleError("IndexError: bed line with fewer than 4 columns");
        std::string arm = col[3];
        const std::string key = col[0] + "_" + arm;
        const std::pair<int64_t, int64_t> v(std::stoll(col[1]), std::stoll(col[2]));
        if (auto* p = table.find(key)) *p = v;
        else table.insert(key, v);
    }
    for (const std::string& k : table.keys()) {
        Region r;
        r.key = k;
        r.chrom = k.substr(0, k.rfind('_'));
        r.start = table.find(k)->first;
        r.end = table.find(k)->second;
        out.push_back(r);
    }
    return out;
}

// the records read_bam sees for one region: fetch (overlap: pos < end and reaching past start) then
// its start <= pos <= end filter, i.e. start <= pos < end on the contig, in file order.  A
// coordinate-sorted file (an indexed fetch, as pysam needs) is searched by bisection.
std::vector<int32_t> fetch(const Bam& b, const Region& rg) {
    std::vector<int32_t> out;
    if (rg.whole) {
        out.resize(b.recs.size());
        for (size_t i = 0; i < out.size(); ++i) out[i] = (int32_t)i;
        return out;
    }
    const int32_t t = b.h.tid(rg.chrom);
    if (t < 0) throw OracleError("ValueError: invalid contig `" + rg.chrom + "`");
    auto key = [](const Rec& r) { return ((uint64_t)(uint32_t)r.tid << 32) | (uint32_t)r.pos; };
    if (b.sorted < 0) {
        bool srt = true;
        for (size_t i = 1; i < b.recs.size() && srt; ++i) srt = key(b.recs[i - 1]) <= key(b.recs[i]);
        const_cast<Bam&>(b).sorted = srt ? 1 : 0;
    }
    const bool sorted = b.sorted == 1;
    size_t lo = 0, hi = b.recs.size();
    if (sorted) {
        const uint64_t k0 = ((uint64_t)(uint32_t)t << 32) | (uint32_t)std::max<int64_t>(rg.start, 0);
        lo = std::lower_bound(b.recs.begin(), b.recs.end(), k0,
                              [&](const Rec& r, uint64_t k) { return key(r) < k; }) - b.recs.begin();
    }
    for (size_t i = lo; i < hi; ++i) {
        const Rec& r = b.recs[i];
        if (sorted && (r.tid != t || r.pos >= rg.end)) break;
        if (r.tid != t || r.pos >= rg.end) continue;
        if (r.endpos() <= rg.start) continue;
        if (r.pos < rg.start || r.pos > rg.end) continue;
        out.push_back((int32_t)i);
    }
    return out;
}

struct Counts {
    int64_t total = 0, mate = 0, multi = 0, spacer = 0;
};

// Members are record indices into the stage's decoded file (a pysam fetch makes a new object per
// record, so equality is by content, pysam's __eq__; the SSCS singleton rename copies the record).
using Fam = std::vector<int32_t>;
struct FamilyBuilder {
    const Bam* bam = nullptr;
    OrderedMap<Fam> pending;                        // pair_dict
    OrderedMap<Fam> members;                        // read_dict
    OrderedMap<int64_t> size;                       // tag_dict
    OrderedMap<std::vector<std::string>> entries;   // csn_pair_dict
    explicit FamilyBuilder(const Bam* b) : bam(b) {}
    const Rec& rec(int32_t i) const { return bam->recs[i]; }

    Counts feed(const std::vector<int32_t>& idx, const char* delim, bool duplex, std::vector<int32_t>* bad) {
        Counts c;
        for (int32_t i : idx) {
            const Rec& r = rec(i);
            c.total += 1;
            bool badr = true;
            if (delim && r.qname.find(delim) == std::string::npos) c.spacer += 1;
            else if (r.is_unmapped()) { c.total -= 1; }
            else if (r.flag == 73 || r.flag == 89 || r.flag == 121 || r.flag == 153 || r.flag == 185 || r.flag == 137)
                c.mate += 1;
            else if (r.flag & 0x100) c.multi += 1;
            else if (r.flag & 0x800) c.multi += 1;
            else badr = false;
            if (badr && bad) { bad->push_back(i); continue; }
            Fam& waiting = pending.get_or_insert(r.qname);
            waiting.push_back(i);
            if (waiting.size() < 2) continue;
            const int32_t fi = waiting[0], si = waiting[1];
            const Rec& first = rec(fi);
            const Rec& second = rec(si);
            std::string barcode;
            if (duplex) barcode = first.qname.substr(0, first.qname.find('_'));
            else {
                const std::vector<std::string> s = split(first.qname, delim ? delim : "|");
                if (s.size() < 2) throw OracleError("IndexError: qname without barcode");
                barcode = s[1];
            }
            const std::string cig = ordered_cigars(first, second);
            const std::string mol = molecule_name(first, second, barcode, cig);
            for (int k = 0; k < 2; ++k) {
                const int32_t ri = k ? si : fi;
                const std::string key = read_end_key(rec(ri), barcode, cig);
                if (!members.has(key) && !size.has(key)) {
                    members.insert(key, Fam{ri});
                    size.get_or_insert(key) += 1;
                    std::vector<std::string>* ent = entries.find(mol);
                    if (!ent) entries.insert(mol, std::vector<std::string>{key});
                    else if (ent->size() < 2) ent->push_back(key);   // else "Consensus tag NOT UNIQUE"
                } else if (size.has(key)) {
                    Fam* fam = members.find(key);
                    if (!fam) throw OracleError("KeyError: " + key + " (read_dict entry already written)");
                    bool in = false;
                    for (int32_t m : *fam)
                        if (m == fi || same_content(rec(m), first)) { in = true; break; }
                    if (!in) {
                        fam->push_back(ri);
                        *size.find(key) += 1;
                    }
                }   // else "line read twice": dropped
            }
            pending.erase(r.qname);
        }
        return c;
    }
    std::vector<const Rec*> recs_of(const Fam& f) const {
        std::vector<const Rec*> v;
        v.reserve(f.size());
        for (int32_t i : f) v.push_back(&rec(i));
        return v;
    }
};

// ------------------------------------------------------------------ votes and records
template <typename T>
T most_common_first(const std::vector<T>& v) {
    std::vector<std::pair<T, int>> cnt;
    for (const T& x : v) {
        bool found = false;
        for (auto& p : cnt)
            if (p.first == x) { ++p.second; found = true; break; }
        if (!found) cnt.push_back({x, 1});
    }
    int top = 0;
    for (auto& p : cnt) top = std::max(top, p.second);
    for (auto& p : cnt)
        if (p.second == top) return p.first;
    return v[0];
}

// Counter over the values: large families use a hash map (same first-seen order)
template <typename T>
T mode_fast(const std::vector<T>& v) {
    if (v.size() <= 16) return most_common_first(v);
    std::unordered_map<T, std::pair<int, size_t>> c;   // count, first index
    for (size_t i = 0; i < v.size(); ++i) {
        auto it = c.find(v[i]);
        if (it == c.end()) c[v[i]] = {1, i};
        else ++it->second.first;
    }
    int top = 0;
    size_t first = 0;
    for (auto& kv : c)
        if (kv.second.first > top || (kv.second.first == top && kv.second.second < first)) {
            top = kv.second.first;
            first = kv.second.second;
        }
    return v[first];
}

int pick_flag(const std::vector<const Rec*>& m) {
    std::vector<int> f;
    for (const Rec* r : m) f.push_back(r->flag);
    std::unordered_map<int, std::pair<int, size_t>> c;
    for (size_t i = 0; i < f.size(); ++i) {
        auto it = c.find(f[i]);
        if (it == c.end()) c[f[i]] = {1, i};
        else ++it->second.first;
    }
    int top = 0;
    for (auto& kv : c) top = std::max(top, kv.second.first);
    std::vector<std::pair<size_t, int>> best;
    for (auto& kv : c)
        if (kv.second.first == top) best.push_back({kv.second.second, kv.first});
    std::sort(best.begin(), best.end());
    if (best.size() == 1) return best[0].second;
    for (int p : {99, 83, 147, 163})
        for (auto& b : best)
            if (b.second == p) return p;
    return best[0].second;
}

Rec new_record(const std::vector<const Rec*>& members, const std::string& seq, const std::string& quals,
               const std::string& name) {
    const Rec& t = *members[0];
    Rec r;
    r.qname = name;
    r.seq = seq;
    r.tid = t.tid;
    r.pos = t.pos;
    std::vector<int> mq, tl;
    for (const Rec* m : members) { mq.push_back(m->mapq); tl.push_back(m->tlen); }
    r.mapq = (uint8_t)mode_fast(mq);
    r.cigar = t.cigar;
    r.mtid = t.mtid;
    r.mpos = t.mpos;
    r.tlen = mode_fast(tl);
    r.qual = quals;
    r.qual_missing = seq.empty();
    r.flag = (uint16_t)pick_flag(members);
    std::vector<std::string> rgs;
    bool all = true;
    for (const Rec* m : members) {
        std::string v;
        char ty;
        if (!m->get_rg(v, ty)) { all = false; break; }
        rgs.push_back(v);
    }
    if (all) {
        const std::string v = mode_fast(rgs);
        r.aux = std::string("RGZ") + v + std::string(1, '\0');
    }
    const int32_t b0 = std::max(r.pos, 0);
    r.bin = (uint16_t)reg2bin(b0, std::max(r.endpos(), b0 + 1));
    return r;
}

void single_strand_vote(const std::vector<const Rec*>& fam, double cutoff, std::string& out_s, std::string& out_q) {
    const int L = fam[0]->infer_query_length();
    if (L < 0) throw OracleError("TypeError: no cigar");
    const int n = (int)fam.size();
    out_s.assign(L, 'N');
    out_q.assign(L, '\0');
    static const char BO[] = "ACGTN";
    struct Idx {   // magic static: initialised once, thread-safe (oracle stages may run on threads)
        int8_t v[256];
        Idx() {
            for (int c = 0; c < 256; ++c) v[c] = -1;
            for (int b = 0; b < 5; ++b) v[(uint8_t)BO[b]] = (int8_t)b;
        }
    };
    static const Idx table;
    const int8_t* idx = table.v;
    for (const Rec* m : fam)
        if (L > 0 && m->qual_missing) throw OracleError("TypeError: qualities missing");
    for (int i = 0; i < L; ++i) {
        int cnt[5] = {0, 0, 0, 0, 0}, qsum[5] = {0, 0, 0, 0, 0}, failed = 0;
        for (const Rec* m : fam) {
            if (i >= (int)m->qual.size() || i >= (int)m->seq.size()) throw OracleError("IndexError: read shorter than consensus");
            const int b = idx[(uint8_t)m->seq[i]];
            if (b < 0) throw OracleError(std::string("ValueError: base ") + m->seq[i]);
            const int q = (uint8_t)m->qual[i];
            if (q < 30) failed += 1;
            else {
                if (b == 4) throw OracleError("IndexError: N with quality >= 30");
                cnt[b] += 1;
                qsum[b] += q;
            }
        }
        int k = 0;
        for (int b = 1; b < 5; ++b)
            if (cnt[b] > cnt[k]) k = b;
        const int mq = std::min(60, qsum[k]);
        const int passed = n - failed;
        if (passed && (double)cnt[k] / (double)passed >= cutoff) out_s[i] = BO[k];
        out_q[i] = (char)mq;
    }
}

void pair_vote(const Rec& a, const Rec& b, bool gate, std::string& out_s, std::string& out_q) {
    const std::string& sa = a.seq;
    const std::string& sb = b.seq;
    const int L = (int)sa.size();
    out_s.assign(L, 'N');
    out_q.assign(L, '\0');
    for (int i = 0; i < L; ++i) {
        if (i >= (int)sb.size()) throw OracleError("IndexError: complement shorter");
        const bool same = sa[i] == sb[i];
        if (same && (a.qual_missing || b.qual_missing)) throw OracleError("TypeError: qualities missing");
        if (same) {
            const int qa = (uint8_t)a.qual[i], qb = (uint8_t)b.qual[i];
            if (!gate || (qa > 29 && qb > 29)) {
                out_s[i] = sa[i];
                out_q[i] = (char)std::min(60, qa + qb);
            }
        }
    }
}

std::string duplex_name(const std::string& tag, const std::string& ds) {
    const std::string bc = tag.substr(0, tag.find('_')), dbc = ds.substr(0, ds.find('_'));
    const std::string rest = tag.substr(tag.find('_') + 1);
    const std::string coords = rest.substr(0, rest.rfind('_'));
    const std::string n_tag = split(tag, ":").at(1), n_ds = split(ds, ":").at(1);
    if (tag.find("pos") != std::string::npos) return bc + "_" + dbc + "_" + coords + ":" + n_tag + "_" + n_ds;
    return dbc + "_" + bc + "_" + coords + ":" + n_ds + "_" + n_tag;
}

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Python float repr (shortest round trip; exponent form outside [1e-4, 1e16))
std::string py_float(double x) {
    if (x == 0) return std::signbit(x) ? "-0.0" : "0.0";
    char buf[64];
    int prec = 1;
    for (; prec <= 17; ++prec) {
        snprintf(buf, sizeof(buf), "%.*e", prec - 1, x);
        if (strtod(buf, nullptr) == x) break;
    }
    // digits and exponent of the shortest form
    std::string s(buf);
    const size_t e = s.find('e');
    const int exp = atoi(s.c_str() + e + 1);
    std::string mant = s.substr(0, e);
    const bool neg = mant[0] == '-';
    if (neg) mant = mant.substr(1);
    std::string digits;
    for (char c : mant)
        if (c != '.') digits.push_back(c);
    std::string out;
    if (exp < -4 || exp >= 16) {
        out = digits.substr(0, 1);
        if (digits.size() > 1) out += "." + digits.substr(1);
        char eb[16];
        snprintf(eb, sizeof(eb), "e%c%02d", exp < 0 ? '-' : '+', std::abs(exp));
        out += eb;
    } else if (exp < 0) {
        out = "0." + std::string(-exp - 1, '0') + digits;
    } else {
        if ((int)digits.size() <= exp + 1) out = digits + std::string(exp + 1 - digits.size(), '0') + ".0";
        else out = digits.substr(0, exp + 1) + "." + digits.substr(exp + 1);
    }
    return neg ? "-" + out : out;
}

void append_text(const std::string& path, const std::string& text, bool truncate) {
    std::ofstream f(path, truncate ? std::ios::trunc : std::ios::app);
    f << text;
}

// ------------------------------------------------------------------ stages
void sscs_stage(const std::string& infile, const std::string& outfile, double cutoff, const char* bedfile,
                const char* bdelim, double* t_cons) {
    Bam bam = read_bam(infile);
    const std::string prefix = outfile.substr(0, outfile.find(".sscs"));
    const double t0 = now();
    std::vector<Rec> sscs_out, single_out;
    std::vector<int32_t> bad_idx;
    FamilyBuilder fb(&bam);
    Counts tot;
    const char* delim = bdelim ? bdelim : "|";
    for (const Region& rg : regions_of(bedfile)) {
        const Counts c = fb.feed(fetch(bam, rg), delim, false, &bad_idx);
        tot.total += c.total; tot.mate += c.mate; tot.multi += c.multi; tot.spacer += c.spacer;
        fb.entries.walk([&](const std::string& mol_ref) {
            const std::string mol = mol_ref;
            std::vector<std::string> keys = *fb.entries.find(mol);
            if (keys.size() != 2) return;
            for (const std::string& k : keys) {
                const Fam& fi = *fb.members.find(k);
                const int64_t n = *fb.size.find(k);
                const std::string name = mol + ":" + std::to_string(n);
                if (n == 1) {
                    Rec r = bam.recs[fi[0]];
                    r.qname = name;
                    r.raw.clear();
                    single_out.push_back(std::move(r));
                } else {
                    const std::vector<const Rec*> fam = fb.recs_of(fi);
                    std::string s, q;
                    single_strand_vote(fam, cutoff, s, q);
                    sscs_out.push_back(new_record(fam, s, q, name));
                }
                fb.members.erase(k);
            }
            fb.entries.erase(mol);
        });
    }
    std::vector<Rec> bad;
    bad.reserve(bad_idx.size());
    for (int32_t i : bad_idx) bad.push_back(bam.recs[i]);
    if (t_cons) *t_cons = now() - t0;
    write_bam(outfile, bam.h, sscs_out);
    write_bam(prefix + ".singleton.bam", bam.h, single_out);
    write_bam(prefix + ".badReads.bam", bam.h, bad);
    append_text(prefix + ".stats.txt",
                "# === SSCS ===\nUncollapsed - Total reads: " + std::to_string(tot.total) +
                    "\nUncollapsed - Unmapped reads: " + std::to_string(tot.mate) +
                    "\nUncollapsed - Secondary/Supplementary reads: " + std::to_string(tot.multi) +
                    "\nSSCS reads: " + std::to_string(sscs_out.size()) + "\nSingletons: " +
                    std::to_string(single_out.size()) + "\nBad spacers: " + std::to_string(tot.spacer) + "\n",
                true);
    // Counter(tag_dict.values()) in first-seen order (SSCS_maker.py:401-408)
    std::vector<std::pair<int64_t, int64_t>> freq;
    std::unordered_map<int64_t, size_t> at;
    for (size_t i = 0; i < fb.size.items.size(); ++i) {
        if (!fb.size.live[i]) continue;
        const int64_t v = fb.size.items[i].second;
        auto it = at.find(v);
        if (it == at.end()) { at[v] = freq.size(); freq.push_back({v, 1}); }
        else freq[it->second].second += 1;
    }
    std::string txt = "family_size\tfrequency\n";
    for (size_t i = 0; i < freq.size(); ++i)
        txt += (i ? "\n" : "") + std::to_string(freq[i].first) + "\t" + std::to_string(freq[i].second);
    append_text(prefix + ".read_families.txt", txt, true);
    if (freq.empty()) throw OracleError("IndexError: empty family table (SSCS_maker.py:417)");
}

void dcs_stage(const std::string& infile, const std::string& outfile, const char* bedfile, double* t_cons) {
    Bam bam = read_bam(infile);
    std::string single_path, title, sc;
    if (outfile.find(".dcs.sc") != std::string::npos) {
        single_path = outfile.substr(0, outfile.find(".dcs.sc")) + ".sscs.sc.singleton.bam";
        title = "DCS - Singleton Correction";
        sc = " SC";
    } else {
        single_path = outfile.substr(0, outfile.find(".dcs")) + ".sscs.singleton.bam";
        title = "DCS";
    }
    const std::string prefix = outfile.substr(0, outfile.find(".dcs"));
    const double t0 = now();
    FamilyBuilder fb(&bam);
    std::unordered_set<std::string> used;   // duplex_dict
    std::vector<Rec> dcs_out, single_out;
    Counts tot;
    for (const Region& rg : regions_of(bedfile)) {
        const Counts c = fb.feed(fetch(bam, rg), nullptr, true, nullptr);
        tot.total += c.total; tot.mate += c.mate;
        fb.entries.walk([&](const std::string& mol_ref) {
            const std::string mol = mol_ref;
            const std::vector<std::string> keys = *fb.entries.find(mol);
            for (const std::string& k : keys) {
                const std::string partner = complement_key(k);
                if (used.count(partner)) continue;
                if (fb.size.has(k) && fb.size.has(partner)) {
                    const Fam* pf = fb.members.find(partner);
                    if (!pf) throw OracleError("KeyError: " + partner);
                    const Rec& a = bam.recs[(*fb.members.find(k))[0]];
                    const Rec& b = bam.recs[(*pf)[0]];
                    std::string s, q;
                    pair_vote(a, b, false, s, q);
                    dcs_out.push_back(new_record({&a, &b}, s, q, duplex_name(a.qname, b.qname)));
                    used.insert(k);
                } else {
                    single_out.push_back(bam.recs[(*fb.members.find(k))[0]]);
                }
                fb.members.erase(k);
            }
            fb.entries.erase(mol);
        });
    }
    if (t_cons) *t_cons = now() - t0;
    write_bam(outfile, bam.h, dcs_out);
    write_bam(single_path, bam.h, single_out);
    append_text(prefix + ".stats.txt",
                "# === " + title + " ===\nSSCS" + sc + " - Total reads: " + std::to_string(tot.total) + "\nSSCS" + sc +
                    " - Unmapped reads: " + std::to_string(tot.mate) + "\nSSCS" + sc +
                    " - Secondary/Supplementary reads: 0\nDCS" + sc + " reads: " + std::to_string(dcs_out.size()) +
                    "\nSSCS" + sc + " singletons: " + std::to_string(single_out.size()) + " \n",
                false);
}

void sc_stage(const std::string& singleton, const char* bedfile, double* t_cons) {
    const size_t cut = singleton.find(".singleton");
    const std::string base = singleton.substr(0, cut), rest = singleton.substr(cut + 10);
    Bam sbam = read_bam(singleton);
    Bam xbam = read_bam(base + ".sscs" + rest);
    const double t0 = now();
    FamilyBuilder singles(&sbam);
    std::unique_ptr<FamilyBuilder> sscs(new FamilyBuilder(&xbam));
    OrderedMap<std::string> resolved;   // correction_dict
    std::vector<Rec> by_sscs, by_single, uncorrected;
    int64_t n_single_reads = 0, n_processed = 0;
    std::string chrom_seen = "chrM";
    for (const Region& rg : regions_of(bedfile)) {
        if (!rg.whole && rg.chrom != chrom_seen) {
            singles.size.clear();
            sscs.reset(new FamilyBuilder(&xbam));
            chrom_seen = rg.chrom;
        }
        n_single_reads += singles.feed(fetch(sbam, rg), nullptr, true, nullptr).total;
        sscs->feed(fetch(xbam, rg), nullptr, true, nullptr);
        singles.entries.walk([&](const std::string& mol_ref) {
            const std::string mol = mol_ref;
            const std::vector<std::string> keys = *singles.entries.find(mol);
            for (const std::string& k : keys) {
                n_processed += 1;
                const std::string partner = complement_key(k);
                const std::string name = mol + ":1";
                const Fam* ownf = singles.members.find(k);
                if (!ownf) throw OracleError("KeyError: " + k);
                const Rec& own = sbam.recs[(*ownf)[0]];
                std::string s, q;
                if (const Fam* xf = sscs->members.find(partner)) {
                    pair_vote(own, xbam.recs[(*xf)[0]], true, s, q);
                    by_sscs.push_back(new_record({&own}, s, q, name));
                    sscs->members.erase(partner);
                    singles.members.erase(k);
                } else if (const Fam* pf = singles.members.find(partner)) {
                    pair_vote(own, sbam.recs[(*pf)[0]], true, s, q);
                    by_single.push_back(new_record({&own}, s, q, name));
                    if (auto* v = resolved.find(k)) *v = partner;
                    else resolved.insert(k, partner);
                    if (resolved.has(partner)) {
                        singles.members.erase(k);
                        singles.members.erase(partner);
                        resolved.erase(k);
                        resolved.erase(partner);
                    }
                } else {
                    uncorrected.push_back(own);
                    singles.members.erase(k);
                }
            }
            singles.entries.erase(mol);
        });
    }
    if (t_cons) *t_cons = now() - t0;
    write_bam(base + ".sscs.correction.bam", sbam.h, by_sscs);
    write_bam(base + ".singleton.correction.bam", sbam.h, by_single);
    write_bam(base + ".uncorrected.bam", sbam.h, uncorrected);
    if (n_single_reads == 0) throw OracleError("ZeroDivisionError: empty singleton file");
    append_text(base + ".stats.txt",
                "# === Singleton Correction ===\nTotal singletons: " + std::to_string(n_processed) +
                    "\nSingleton Correction by SSCS: " + std::to_string(by_sscs.size()) +
                    "\n% Singleton Correction by SSCS: " + py_float((double)by_sscs.size() / (double)n_single_reads * 100) +
                    "\nSingleton Correction by Singletons: " + std::to_string(by_single.size()) +
                    "\n% Singleton Correction by Singletons : " +
                    py_float((double)by_single.size() / (double)n_single_reads * 100) +
                    "\nUncorrected Singletons: " + std::to_string(uncorrected.size()) + " \n",
                false);
}

uint64_t sort_key(const Rec& r) {
    return ((uint64_t)(uint32_t)r.tid << 32) | ((uint64_t)((uint32_t)(r.pos + 1)) << 1) | ((r.flag >> 4) & 1u);
}

// canonical per-record digest: every field pysam compares, aux tags in sorted order (bin excluded)
uint64_t digest(const Rec& r) {
    Rec c = r;
    std::vector<std::string> tags;
    size_t p = 0;
    while (p + 3 <= r.aux.size()) {
        const char typ = r.aux[p + 2];
        size_t q = p + 3, vlen = 0;
        switch (typ) {
            case 'A': case 'c': case 'C': vlen = 1; break;
            case 's': case 'S': vlen = 2; break;
            case 'i': case 'I': case 'f': vlen = 4; break;
            case 'Z': case 'H': vlen = r.aux.find('\0', q) - q + 1; break;
            case 'B': {
                const char sub = r.aux[q];
                const uint32_t cnt = rdu32(r.aux.data() + q + 1);
                vlen = 5 + cnt * ((sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4);
                break;
            }
            default: vlen = r.aux.size() - q;
        }
        tags.push_back(r.aux.substr(p, 3 + vlen));
        p = q + vlen;
    }
    std::sort(tags.begin(), tags.end());
    c.aux.clear();
    for (auto& t : tags) c.aux += t;
    hash_content(c);
    return c.content;
}

}  // namespace

// ================================================================== C ABI (test infrastructure)
extern "C" {

const char* ccor_last_error() { return g_err.c_str(); }

#define CCOR_TRY(...)                                   \
    try {                                               \
        __VA_ARGS__;                                    \
        return 0;                                       \
    } catch (const std::exception& e) {                 \
        g_err = e.what();                               \
        return -1;                                      \
    }

int ccor_sscs(const char* infile, const char* outfile, double cutoff, const char* bedfile, const char* bdelim,
              double* t_cons) {
    CCOR_TRY(sscs_stage(infile, outfile, cutoff, bedfile, bdelim, t_cons))
}
int ccor_dcs(const char* infile, const char* outfile, const char* bedfile, double* t_cons) {
    CCOR_TRY(dcs_stage(infile, outfile, bedfile, t_cons))
}
int ccor_sc(const char* singleton, const char* bedfile, double* t_cons) {
    CCOR_TRY(sc_stage(singleton, bedfile, t_cons))
}
// samtools sort stand-in: X.bam -> X.sorted.bam (stable on tid<<32 | (pos+1)<<1 | rev), X.bam removed
int ccor_sort(const char* in_path, const char* out_path) {
    CCOR_TRY({
        Bam b = read_bam(in_path);
        std::vector<std::pair<uint64_t, size_t>> key(b.recs.size());
        for (size_t i = 0; i < key.size(); ++i) key[i] = {sort_key(b.recs[i]), i};
        std::sort(key.begin(), key.end());   // (key, input index): the stable order
        std::vector<Rec> recs(key.size());
        for (size_t i = 0; i < key.size(); ++i) recs[i] = std::move(b.recs[key[i].second]);
        write_bam(out_path, b.h, recs);
        std::remove(in_path);
    })
}
// samtools merge stand-in: ties in input-file order
int ccor_merge(const char* out_path, const char* const* in_paths, int n) {
    CCOR_TRY({
        Header h;
        std::vector<std::pair<std::pair<uint64_t, std::pair<int, size_t>>, Rec>> all;
        for (int i = 0; i < n; ++i) {
            Bam b = read_bam(in_paths[i]);
            if (i == 0) h = b.h;
            for (size_t k = 0; k < b.recs.size(); ++k)
                all.push_back({{sort_key(b.recs[k]), {i, k}}, std::move(b.recs[k])});
        }
        std::sort(all.begin(), all.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        std::vector<Rec> recs;
        recs.reserve(all.size());
        for (auto& x : all) recs.push_back(std::move(x.second));
        write_bam(out_path, h, recs);
    })
}
// per-record canonical digests in file order (tests compare files with them); returns the count
int64_t ccor_digests(const char* path, uint64_t* out, int64_t cap) {
    try {
        Bam b = read_bam(path);
        const int64_t n = (int64_t)b.recs.size();
        if (out) parallel_for((size_t)std::min(n, cap), [&](size_t i) { out[i] = digest(b.recs[i]); });
        return n;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}
int ccor_py_float(double x, char* buf, int cap) {
    snprintf(buf, cap, "%s", py_float(x).c_str());
    return 0;
}

}  // extern "C"
