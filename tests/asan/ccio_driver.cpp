// Host sanitizer driver (ASan/UBSan on the C++ library).  Built with
// -fsanitize=address,undefined together with consensuscruncher_amd/csrc/ccio.cpp by
// tests/test_ccio_asan.py; exercises every libccio entry point the stages use on a BAM file:
// open, layout, decode (both barcode modes), the interner and its swap table, record writing
// (raw, renamed and new records), sort, merge, concat, index and the name formatters; with two
// FASTQ arguments also the UMI extraction (pattern and list modes, one and several threads).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/consensuscruncher_amd.h"

static int fail(const char* what) {
    fprintf(stderr, "FAIL %s: %s\n", what, ccio_last_error());
    return 1;
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const std::string in = argv[1], dir = argv[2], sscs = argv[3];
    for (int mode = 0; mode < 2; ++mode) {
        ccio_bam* b = ccio_bam_open(in.c_str(), 2);
        if (!b) return fail("open");
        const int64_t n = ccio_bam_nrec(b);
        uint64_t qnb = 0, pb = 0;
        int32_t ml = 0;
        if (ccio_bam_layout(b, &qnb, &pb, &ml, 2)) return fail("layout");
        std::vector<int32_t> tid(n), pos(n), mtid(n), mpos(n), tlen(n), cig(n), qlen(n), lseq(n), bc(n), rg(n);
        std::vector<uint16_t> flag(n), qn_len(n);
        std::vector<uint8_t> mapq(n), rflags(n), qn_blob(qnb + 16), payload(pb + 64);
        std::vector<uint64_t> qn_off(n), pay_off(n), rdig(n);
        cc_records r;
        memset(&r, 0, sizeof r);
        r.n = n; r.tid = tid.data(); r.pos = pos.data(); r.mtid = mtid.data(); r.mpos = mpos.data(); r.tlen = tlen.data();
        r.flag = flag.data(); r.mapq = mapq.data(); r.cigar_id = cig.data(); r.qlen = qlen.data(); r.lseq = lseq.data();
        r.bc_id = bc.data(); r.rg_id = rg.data(); r.rflags = rflags.data(); r.qn_off = qn_off.data(); r.qn_len = qn_len.data();
        r.qn_blob = qn_blob.data(); r.qn_blob_bytes = qnb; r.pay_off = pay_off.data(); r.payload = payload.data();
        r.payload_bytes = pb; r.rdig = rdig.data();
        ccio_interner* it = ccio_interner_new();
        if (ccio_bam_decode(b, it, mode, "|", &r, 2)) return fail("decode");
        const int64_t ns = ccio_interner_swap_table(it, nullptr, 0);
        std::vector<int32_t> swap(ns > 0 ? ns : 1);
        ccio_interner_swap_table(it, swap.data(), ns);
        char buf[512];
        for (int64_t i = 0; i < ccio_interner_size(it, 0); ++i) ccio_interner_get(it, 0, i, buf, sizeof buf);
        // raw, renamed and new records
        std::vector<cc_out_spec> spec(n);
        std::vector<int64_t> noff(n + 1);
        std::string names;
        std::vector<uint8_t> cseq((size_t)n * 128 + 64, 0x11), cqual((size_t)n * 256 + 64, 35);
        for (int64_t i = 0; i < n; ++i) {
            memset(&spec[i], 0, sizeof(cc_out_spec));
            spec[i].kind = (int32_t)(i % 3);
            spec[i].src_rec = i;
            spec[i].name_id = i;
            spec[i].rg_id = -1;
            spec[i].flag = flag[i];
            spec[i].mapq = 60;
            spec[i].cons_len = lseq[i] < 200 ? lseq[i] : 200;
            spec[i].cons_off = i * 256;
            noff[i] = (int64_t)names.size();
            names += "name" + std::to_string(i);
        }
        noff[n] = (int64_t)names.size();
        ccio_bam* srcs[1] = {b};
        const std::string w = dir + "/w" + std::to_string(mode) + ".bam";
        if (ccio_write_bam(w.c_str(), b, it, n, spec.data(), srcs, 1, names.data(), noff.data(), cseq.data(),
                           cqual.data(), 1, 2))
            return fail("write");
        const std::string s = dir + "/s" + std::to_string(mode) + ".bam";
        if (ccio_sort_bam(w.c_str(), s.c_str(), 1, 2)) return fail("sort");
        if (ccio_index_bam(s.c_str())) return fail("index");
        const char* ins[2] = {s.c_str(), in.c_str()};
        const std::string m = dir + "/m" + std::to_string(mode) + ".bam";
        if (ccio_merge_bams(m.c_str(), ins, 2, 1, 2)) return fail("merge");
        const std::string c = dir + "/c" + std::to_string(mode) + ".bam";
        if (ccio_concat_bams(c.c_str(), ins, 2, 1, 2)) return fail("concat");
        // rank-local record sets: BAI region reads, cores, pack, combine (sorted two ways), write
        {
            const int32_t rt[3] = {0, 0, 1};
            const int64_t rb[3] = {0, 5000, 0}, re[3] = {3000, 1 << 28, 1 << 28};
            ccio_bam* sub = ccio_bam_open_regions(s.c_str(), 3, rt, rb, re, 2);
            if (!sub) return fail("open_regions");
            const int64_t k = ccio_bam_nrec(sub);
            std::vector<int32_t> t(k + 1), p(k + 1), mt(k + 1), mp(k + 1);
            std::vector<uint16_t> fl(k + 1);
            ccio_bam_cores(sub, t.data(), p.data(), mt.data(), mp.data(), fl.data());
            std::vector<int64_t> idx;
            for (int64_t i = k - 1; i >= 0; i -= 2) idx.push_back(i);
            const int64_t nb = ccio_bam_pack(sub, (int64_t)idx.size(), idx.data(), nullptr, 0);
            if (nb < 0) return fail("pack size");
            std::vector<uint8_t> blob(nb + 1);
            if (ccio_bam_pack(sub, (int64_t)idx.size(), idx.data(), blob.data(), nb) != nb) return fail("pack");
            const uint8_t* blobs[1] = {blob.data()};
            const int64_t bn[1] = {nb};
            ccio_bam* parts[1] = {sub};
            for (int key = 0; key < 3; ++key) {
                ccio_bam* cb = ccio_bam_combine(nullptr, parts, 1, blobs, bn, 1, key, 2);
                if (!cb) return fail("combine");
                std::vector<int64_t> org(ccio_bam_nrec(cb) + 1);
                if (ccio_bam_origin(cb, org.data())) return fail("origin");
                if (ccio_bam_write_all((dir + "/cb" + std::to_string(key) + ".bam").c_str(), cb, 1, 2))
                    return fail("write_all");
                ccio_bam_close(cb);
            }
            ccio_bam_close(sub);
            int64_t rbytes[3];
            if (ccio_bai_region_bytes(s.c_str(), 3, rt, rb, re, rbytes)) return fail("region bytes");
            if (ccio_bai_mapped(s.c_str()) < 0) return fail("bai mapped");
        }
        // a truncated BAM: the index and the reader report an error, they do not read past the end
        {
            FILE* fi = fopen(s.c_str(), "rb");
            std::vector<char> all;
            char tmp[4096];
            size_t got;
            while ((got = fread(tmp, 1, sizeof tmp, fi)) > 0) all.insert(all.end(), tmp, tmp + got);
            fclose(fi);
            const std::string tr = dir + "/trunc" + std::to_string(mode) + ".bam";
            FILE* fo = fopen(tr.c_str(), "wb");
            fwrite(all.data(), 1, all.size() / 2, fo);
            fclose(fo);
            (void)ccio_index_bam(tr.c_str());
            ccio_bam* tb = ccio_bam_open(tr.c_str(), 2);
            if (tb) ccio_bam_close(tb);
        }
        ccio_interner_free(it);
        ccio_bam_close(b);
    }
    // dcs_consensus_tag over SSCS records (their qnames carry the consensus tags)
    ccio_bam* x = ccio_bam_open(sscs.c_str(), 2);
    if (!x) return fail("open sscs");
    const int64_t n = ccio_bam_nrec(x);
    std::vector<int64_t> a(n), d(n), off(n + 1);
    for (int64_t i = 0; i < n; ++i) { a[i] = i; d[i] = n - 1 - i; }
    const int64_t need = ccio_format_dcs_names(x, n, a.data(), d.data(), nullptr, 0, off.data());
    if (need < 0) return fail("dcs names size");
    std::vector<char> blob(need + 1);
    if (ccio_format_dcs_names(x, n, a.data(), d.data(), blob.data(), need, off.data()) < 0) return fail("dcs names");
    ccio_bam_close(x);
    if (argc >= 6) {
        int64_t counts[4], n_written = 0;
        std::vector<int64_t> h1(64), h2(64);
        const char* blist[4] = {"TGT", "CCT", "TGTT", "TT"};
        for (int t = 1; t <= 3; t += 2) {
            const std::string pre = dir + "/fq" + std::to_string(t);
            if (ccio_extract_barcodes(argv[4], argv[5], pre.c_str(), "NNT", nullptr, 0, t, counts, h1.data(), h2.data(),
                                      &n_written))
                return fail("extract pattern");
            if (ccio_extract_barcodes(argv[4], argv[5], (pre + "l").c_str(), nullptr, blist, 4, t, counts, h1.data(),
                                      h2.data(), &n_written))
                return fail("extract list");
        }
    }
    printf("ok\n");
    return 0;
}
