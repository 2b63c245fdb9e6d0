/*
 * consensuscruncher_amd.h — C ABI of the MI355X consensus engine.
 *
 * Two shared libraries sit behind this header:
 *
 *   libccio.so  (host C++)  BAM/BGZF codec, SoA packing, output assembly.
 *                            Replaces pysam/htslib as used by the stage scripts
 *                            (consensus_helper.py:25; SSCS_maker.py:233-244;
 *                            DCS_maker.py:162-176; singleton_correction.py:146-164)
 *                            and the samtools sort/merge calls of
 *                            ConsensusCruncher.py:10-34,262-266,299-304.
 *   libccamd.so (HIP, gfx950) the consensus hot path on the GPU:
 *        cc_read_bam            <- consensus_helper.read_bam           (consensus_helper.py:308-506)
 *                                  + which_read/which_strand/cigar_order/sscs_qname/unique_tag (:57-305)
 *        cc_consensus_maker     <- SSCS_maker.consensus_maker + the SSCS region loop
 *                                  (SSCS_maker.py:81-168, 312-339) + create_aligned_segment
 *                                  /read_mode/consensus_flag (consensus_helper.py:509-619)
 *        cc_duplex_consensus    <- DCS_maker main pairing loop + duplex_consensus + duplex_tag
 *                                  (DCS_maker.py:99-123, 245-282; consensus_helper.py:639-683)
 *        cc_singleton_correction<- singleton_correction main loop + duplex_consensus/strand_correction
 *                                  (singleton_correction.py:61-111, 278-319)
 *
 * The reference has no FFI: its boundary is three Python scripts launched by
 * ConsensusCruncher.py consensus (ConsensusCruncher.py:171-185,206-213,230-237,
 * 280-287).  The Python stage scripts in consensuscruncher_amd/ keep those CLIs
 * and call these entry points through ctypes.
 *
 * Conventions: every function returns 0 on success and a negative CC_E_* code
 * on failure (text from cc_last_error / ccio_last_error).  Host buffers are
 * always owned by the caller; device buffers by the context.  No C++ types
 * cross the ABI.
 */
#ifndef CONSENSUSCRUNCHER_AMD_H
#define CONSENSUSCRUNCHER_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ errors */
#define CC_OK 0
#define CC_E_INVALID -1        /* bad argument / handle */
#define CC_E_HIP -2            /* HIP runtime error */
#define CC_E_N_HIGHQ -3        /* N base with Q>=30 inside a family of size>=2 (SSCS_maker.py:129 IndexError) */
#define CC_E_BAD_BASE -4       /* base outside A,C,G,T,N in a voted family (SSCS_maker.py:122,127 ValueError) */
#define CC_E_SHORT_READ -5     /* member shorter than the inferred read length (IndexError) */
#define CC_E_NO_QUAL -6        /* qualities absent ('*') in a voted read (TypeError) */
#define CC_E_NO_CIGAR -7       /* infer_query_length() is None (TypeError) */
#define CC_E_DUP_QNAME -8      /* (no longer returned: qnames seen more than twice pair in stream order) */
#define CC_E_AMBIGUOUS -9      /* one consensus tag created in two regions (tags of one pair completing apart) */
#define CC_E_COLLISION -10     /* internal 64-bit hash collision (callers retry with another seed) */
#define CC_E_UNSUPPORTED -11
#define CC_E_KEYERROR -12      /* the reference raises KeyError (DCS_maker.py:258: read_dict[duplex] deleted,
                                  reached with duplex keys that are not mutual) */
#define CC_E_REPLAY -13        /* cc_commit: a deferred planned pass did not hold; run the same calls again
                                  with deferral off */

/* record flags (cc_records.rflags) */
#define CC_RF_BAD_SPACER 1u    /* barcode delimiter absent from qname (consensus_helper.py:408) */
#define CC_RF_QUAL_MISSING 2u  /* BAM qual[0] == 0xff */
#define CC_RF_RG_UNSUPPORTED 4u/* RG tag of a type other than Z/A */

/* ---------------------------------------------------------- record SoA
 * One entry per BAM record, in file order.  The payload blob holds, per
 * record at pay_off[i] (16-byte aligned): qualities (lseq bytes, zero padded to
 * 16) then the BAM 4-bit sequence ((lseq+1)/2 bytes, first base in the high
 * nibble, zero padded to 16).  qn_blob holds each qname in an 8-byte aligned,
 * zero padded slot at qn_off[i].  String fields are exact interned ids
 * (ccio_interner): bc_id (barcode by stage mode, -1 if absent), cigar_id
 * (cigarstring, 'None' interned for no cigar), rg_id (-1 if no RG). */
typedef struct cc_records {
    int64_t n;
    int32_t *tid, *pos, *mtid, *mpos, *tlen;
    uint16_t *flag;
    uint8_t *mapq;
    int32_t *cigar_id, *qlen, *lseq, *bc_id, *rg_id;
    uint8_t *rflags;
    uint64_t *qn_off;
    uint16_t *qn_len;
    uint8_t *qn_blob;
    uint64_t qn_blob_bytes;
    uint64_t *pay_off;
    uint8_t *payload;
    uint64_t payload_bytes;
    uint64_t *rdig;     /* 64-bit digest of the whole record (every byte but bin): record equality,
                           pysam's AlignedSegment.__eq__, for the "line read twice" rule when a qname
                           occurs more than twice (consensus_helper.py:490-500) */
} cc_records;

/* ---------------------------------------------------------- output spec */
#define CC_OUT_RAW 0     /* copy the source record unchanged */
#define CC_OUT_RENAME 1  /* source record with qname replaced (SSCS_maker.py:319-321) */
#define CC_OUT_NEW 2     /* new consensus record on the template (create_aligned_segment) */

typedef struct cc_out_spec {
    int32_t kind;
    int32_t src_file;   /* index into the srcs[] array passed to ccio_write_bam */
    int64_t src_rec;    /* record (template) index in that file */
    int64_t name_id;    /* index into the names blob (kinds 1, 2) */
    int32_t flag, mapq, tlen, rg_id;  /* kind 2 */
    int64_t cons_off;   /* kind 2: qual at cons_qual+cons_off, seq nibbles at cons_seq+cons_off/2 */
    int32_t cons_len;   /* kind 2 */
    int32_t pad;
} cc_out_spec;

/* ================================================================ libccio */
typedef struct ccio_interner ccio_interner;
typedef struct ccio_bam ccio_bam;

const char *ccio_last_error(void);
ccio_interner *ccio_interner_new(void);
void ccio_interner_free(ccio_interner *it);
int64_t ccio_interner_size(ccio_interner *it, int kind);               /* 0 barcode, 1 cigar, 2 RG */
int ccio_interner_get(ccio_interner *it, int kind, int64_t id, char *buf, int buflen);
int32_t ccio_interner_intern(ccio_interner *it, int kind, const char *s);
int64_t ccio_interner_swap_table(ccio_interner *it, int32_t *out, int64_t cap); /* duplex_tag barcode swap */

ccio_bam *ccio_bam_open(const char *path, int nthreads);
void ccio_bam_close(ccio_bam *b);
int64_t ccio_bam_nrec(ccio_bam *b);
int32_t ccio_bam_nref(ccio_bam *b);
int ccio_bam_ref(ccio_bam *b, int32_t i, char *name, int cap, int32_t *len);
int ccio_bam_qname(ccio_bam *b, int64_t i, char *buf, int cap);
int ccio_bam_layout(ccio_bam *b, uint64_t *qn_bytes, uint64_t *pay_bytes, int32_t *max_len, int nthreads);
/* mode 0: SSCS barcode = qname.split(delim)[1]; mode 1: duplex barcode = qname.split('_')[0] */
int ccio_bam_decode(ccio_bam *b, ccio_interner *it, int mode, const char *delim, cc_records *out, int nthreads);

/* sscs_qname fields (9 int32 per name: bc, tidLo, posLo, tidHi, posHi, cigA, cigB,
 * strand(0 pos/1 neg/2 None), |tlen|) + ':' + suffix.  blob NULL = size query. */
int64_t ccio_format_csn_names(ccio_interner *it, int64_t n, const int32_t *f9, const int64_t *suffix,
                              char *blob, int64_t cap, int64_t *off);
int ccio_dcs_name(const char *tag, const char *ds, char *out, int cap);
/* duplex_tag(tag) (consensus_helper.py:639-683): barcode halves swapped around the first '.' (else at
 * len // 2), field 8 R1 <-> R2 (anything but R1 -> R1).  Returns the length (snprintf), -1 for fewer
 * than 9 '_' fields (the reference's IndexError). */
int ccio_duplex_tag(const char *tag, char *out, int cap);
int64_t ccio_format_dcs_names(ccio_bam *b, int64_t n, const int64_t *rec_tag, const int64_t *rec_ds,
                              char *blob, int64_t cap, int64_t *off);
int ccio_write_bam(const char *path, ccio_bam *tmpl, ccio_interner *it, int64_t n, const cc_out_spec *spec,
                   ccio_bam *const *srcs, int nsrc, const char *names, const int64_t *name_off,
                   const uint8_t *cons_seq, const uint8_t *cons_qual, int level, int nthreads);
int ccio_sort_bam(const char *in_path, const char *out_path, int level, int nthreads);
int ccio_merge_bams(const char *out_path, const char *const *in_paths, int nin, int level, int nthreads);
/* Writer flags of the orchestrator's fused steps (ConsensusCruncher.py:10-34 sort_index: the stage
 * output sorted and indexed as it is written, instead of written, re-read, sorted and re-read again
 * for the index).  CCIO_W_SORT: records in samtools-sort order (tid, pos, is_reverse; ties keep the
 * written order); CCIO_W_INDEX: also <path>.bai.  keep (non-null) receives a handle over the written
 * records, as ccio_bam_open(path) would return it. */
#define CCIO_W_SORT 1
#define CCIO_W_INDEX 2
/* CCIO_W_ASYNC: the file (and its index) is compressed and written by a thread of its own after the
 * call returns (the kept handle is usable at once); an entry point reading that path, or writing
 * it again, waits for it first; ccio_flush waits for all and reports the first failure */
#define CCIO_W_ASYNC 4
int ccio_flush(void);
/* per value 0..maxv of v[0..n): count and first index (n when absent), one pass (read_families.txt) */
int ccio_value_census(const int32_t *v, int64_t n, int32_t maxv, int64_t *first, int64_t *count);
int ccio_write_bam_ex(const char *path, ccio_bam *tmpl, ccio_interner *it, int64_t n, const cc_out_spec *spec,
                      ccio_bam *const *srcs, int nsrc, const char *names, const int64_t *name_off,
                      const uint8_t *cons_seq, const uint8_t *cons_qual, int level, int nthreads, int flags,
                      ccio_bam **keep);
int ccio_sort_bam_ex(const char *in_path, const char *out_path, int level, int nthreads, int flags);
/* samtools merge of coordinate-sorted record sets held in memory (ties keep input order) */
int ccio_merge_handles(const char *out_path, ccio_bam *const *ins, int nin, int level, int nthreads, int flags,
                       ccio_bam **keep);
/* records of the inputs in file order, one file after the other (sharded stage parts, rank order) */
int ccio_concat_bams(const char *out_path, const char *const *in_paths, int nin, int level, int nthreads);
/* <path>.bai for a coordinate-sorted BAM (samtools index, ConsensusCruncher.py:10-34) */
int ccio_index_bam(const char *path);
/* fastq2bam's UMI extraction (extract_barcodes.py:144-481; replaces its per-pair loop :287-405).
 * pattern (N = barcode base, A/C/G/T = spacer) or, with pattern NULL, the barcode list blist[nblist]
 * (distinct entries; the reference's --skipcheck path).  Writes <out_prefix>_barcode_R1.fastq and
 * _R2.fastq (list mode also _r1/_r2_bad_barcodes.txt).  counts[4] = read pairs, missing spacer, bad
 * barcodes, passing; r1_hist/r2_hist: pattern mode plen x 5 (A,C,G,T,N per barcode position), list
 * mode one count per list entry; *n_written = pairs written before a stop.  Returns 0, -1 (I/O or
 * FASTQ format), -2 (read ids differ: the reference's AssertionError at :291, earlier pairs written)
 * or -3 (a read shorter than the barcode). */
int ccio_extract_barcodes(const char *read1, const char *read2, const char *out_prefix, const char *pattern,
                          const char *const *blist, int32_t nblist, int nthreads, int64_t *counts,
                          int64_t *r1_hist, int64_t *r2_hist, int64_t *n_written);
/* The same extraction with the per-pair decisions made on the GPU (cc_extract_barcodes): the FASTQs
 * read and indexed, stopping where the reference stops (ids differ at a pair: *stop = -2; pattern
 * mode, a read shorter than min_len: -3); the first `width` bases of each pair's reads; the outputs
 * written from the decisions (status 0: passing, header barcode bc + i * bc_stride (NUL terminated),
 * reads cut by cut1 / cut2; list mode, bad-barcode lines per read mask: bit j the prefix of length
 * min(lens[j], read length), bit 31 that of the last length once more). */
typedef struct ccio_fq ccio_fq;
ccio_fq *ccio_fq_open(const char *read1, const char *read2, int32_t min_len, int nthreads);
void ccio_fq_close(ccio_fq *f);
int ccio_fq_info(ccio_fq *f, int64_t *n, int32_t *stop);
int ccio_fq_heads(ccio_fq *f, int32_t width, uint8_t *h1, uint8_t *h2, int32_t *len1, int32_t *len2);
int ccio_fq_write(ccio_fq *f, const char *out_prefix, int list_mode, const uint8_t *status, const char *bc,
                  int32_t bc_stride, const int32_t *cut1, const int32_t *cut2, const uint32_t *bad1,
                  const uint32_t *bad2, const int32_t *lens, int32_t nlens, int nthreads);
/* rank-local record sets of the multi-GPU driver (consensuscruncher_amd/sharded.py) */
/* records with tid == tid[i] and beg[i] <= pos < end[i] for some region i (pysam region fetch +
 * consensus_helper.py:391-396), file order, each once; only the blocks <path>.bai names are read */
ccio_bam *ccio_bam_open_regions(const char *path, int32_t n, const int32_t *tid, const int64_t *beg,
                                const int64_t *end, int nthreads);
int ccio_bam_cores(ccio_bam *b, int32_t *tid, int32_t *pos, int32_t *mtid, int32_t *mpos, uint16_t *flag);
/* raw records idx[0..n) concatenated, block_size first; out NULL: size query */
int64_t ccio_bam_pack(ccio_bam *b, int64_t n, const int64_t *idx, uint8_t *out, int64_t cap);
/* parts' records, then the blobs' raw records, stably sorted by key (0: tid,pos; 1: samtools sort
 * stand-in tid,pos,is_reverse; 2: none); header from tmpl or parts[0] */
ccio_bam *ccio_bam_combine(ccio_bam *tmpl, ccio_bam *const *parts, int32_t n, const uint8_t *const *blobs,
                           const int64_t *blob_bytes, int32_t nb, int key, int nthreads);
int ccio_bam_origin(ccio_bam *b, int64_t *out);   /* each record's input index in its combine */
int ccio_bam_write_all(const char *path, ccio_bam *b, int level, int nthreads);
int64_t ccio_bai_mapped(const char *path);        /* AlignmentFile.mapped from <path>.bai */
int ccio_bai_region_bytes(const char *path, int32_t n, const int32_t *tid, const int64_t *beg, const int64_t *end,
                          int64_t *out);          /* compressed bytes per region: shard-plan weights */
int ccio_write_columns(const char *path, const char *header_text, int32_t nref, const char *const *ref_names,
                       const int32_t *ref_lens, int64_t n, const int32_t *tid, const int32_t *pos,
                       const int32_t *mtid, const int32_t *mpos, const int32_t *tlen, const uint16_t *flag,
                       const uint8_t *mapq, const uint8_t *qn_blob, const int64_t *qn_off, const int32_t *cig_id,
                       const uint32_t *cig_ops, const int64_t *cig_off, int32_t read_len, const uint8_t *seq_ascii,
                       const uint8_t *qual, const int32_t *rg_id, const char *const *rg_vals, int level,
                       int nthreads);

/* ================================================================ libccamd */
typedef struct cc_ctx cc_ctx;

/* counters written by cc_read_bam (consensus_helper.py:383-387, 506) */
enum {
    CC_CNT_COUNTER = 0,       /* records fetched minus is_unmapped */
    CC_CNT_UNMAPPED,          /* is_unmapped */
    CC_CNT_UNMAPPED_MATE,     /* flag in {73,89,121,153,185,137} */
    CC_CNT_MULTIPLE_MAPPING,  /* secondary + supplementary */
    CC_CNT_BAD_SPACER,
    CC_CNT_PAIRS,             /* completed pairs */
    CC_CNT_READ_ENDS,         /* read ends (2 per pair) */
    CC_CNT_FAMILIES,          /* tags (tag_dict entries) */
    CC_CNT_ENTRIES,           /* csn_pair_dict entries */
    CC_CNT_UNPAIRED,          /* pair_dict leftovers */
    CC_CNT_ORPHAN_TAGS,       /* tags beyond two per consensus tag ("NOT UNIQUE") */
    CC_CNT_DROPPED,           /* "line read twice" drops (tag equal to its mate's tag) */
    CC_CNT_BAD_LISTED,        /* records routed to badReads */
    CC_CNT_FOREIGN,           /* stream entries counted on another shard (moved / foreign entries) */
    CC_NUM_COUNTERS = 16
};

typedef struct cc_read_bam_params {
    int32_t delim_filter;  /* SSCS: qname without delimiter is a bad read */
    int32_t badread_file;  /* 1: filtered records go to badReads and are not paired (SSCS) */
    int32_t scope_by_run;  /* singleton_correction's SSCS side: dicts reset per chromosome run */
    int32_t coord_sorted;  /* table is coordinate-sorted (tid, pos): group tags per position group */
    uint64_t seed;         /* hash seed (retry with another on CC_E_COLLISION) */
} cc_read_bam_params;

int cc_create(int device_id, cc_ctx **ctx);
int cc_destroy(cc_ctx *ctx);
const char *cc_last_error(cc_ctx *ctx);
void *cc_host_alloc(cc_ctx *ctx, uint64_t bytes);   /* pinned host memory */
void cc_host_free(cc_ctx *ctx, void *p);
int cc_set_profiling(cc_ctx *ctx, int on);
/* restrict profiling to the newline-separated kernel scopes in names (NULL or "": all) */
int cc_profile_only(cc_ctx *ctx, const char *names);
/* name, total ms, launches for every profiled kernel: returns count */
int cc_kernel_times(cc_ctx *ctx, char *names, int names_cap, double *ms, int64_t *launches, int cap);
int cc_synchronize(cc_ctx *ctx);
/* Deferred end-of-pass checks (no reference counterpart: the reference has no device).  With
 * deferral on, a stage call that re-runs a planned pass (cc_read_bam_rerun, cc_consensus_maker,
 * cc_duplex_consensus, cc_singleton_correction on a group that ran before) enqueues its check and
 * returns without waiting; cc_commit waits once and returns CC_E_REPLAY when any deferred pass
 * must be re-run (the caller repeats the same calls with deferral off).  Counters and results of
 * deferred passes are valid only after cc_commit returned 0. */
int cc_defer(cc_ctx *ctx, int on);
int cc_commit(cc_ctx *ctx);
/* test hook: shifts one planned total (e.g. "scan_pairs") of a group by delta, so that the group's
 * next planned pass fails its check and re-runs exactly */
int cc_debug_skew_plan(cc_ctx *ctx, int32_t group_id, const char *name, int64_t delta);
/* 1 for the debug build (libccamd_debug.so, compiled with -DCC_DEBUG_BOUNDS): its kernels check record,
 * qname, payload, slot and vote indices against their arrays, replace a bad index by 0 and record the
 * first failure; every call that waits for the device (and cc_synchronize) then returns CC_E_INVALID
 * naming the check.  0 for the release build (no checks). */
int cc_debug_build(void);
/* device operations this process's contexts have enqueued so far (kernel launches, memsets, async
 * copies; a rocPRIM sort counts once): the difference over a step is its launch count */
int64_t cc_launch_count(void);

/* copy a record SoA into HBM; returns a table id */
int cc_table_upload(cc_ctx *ctx, const cc_records *rec, int32_t max_len, int32_t *table_id);
int cc_table_free(cc_ctx *ctx, int32_t table_id);

/* read_bam over a record stream (region-major order; stream_rec indexes the
 * table, stream_region gives the region of each stream position,
 * region_run[r] the chromosome-run id of region r).  Multi-GPU sharding: a
 * first-streamed end whose pair completes on another shard is MOVED there.  On
 * the receiver it is a foreign entry, region -(r+1): it pairs and is counted
 * there, is never listed as a bad read, and is neither paired nor counted when
 * it is a bad read of a pass that lists them.  On the sender it keeps its own
 * entry with region r | CC_REGION_MOVED: never paired, counted and listed only
 * as such a bad read.  Each record is thus counted once over the shards.
 * CC_CNT_FOREIGN counts the entries not counted here.  Produces a group id. */
#define CC_REGION_MOVED (1 << 30)
int cc_read_bam(cc_ctx *ctx, int32_t table_id, int64_t n_stream, const int32_t *stream_rec,
                const int32_t *stream_region, int32_t n_regions, const int32_t *region_run,
                const cc_read_bam_params *params, int32_t *group_id);
int cc_group_counters(cc_ctx *ctx, int32_t group_id, int64_t *counters /* CC_NUM_COUNTERS */);
int cc_group_free(cc_ctx *ctx, int32_t group_id);

/* SSCS: consensus_maker over every family emitted by the region loop.  The
 * cutoff test count/pass >= cutoff is evaluated in IEEE double on the GPU,
 * exactly as Python evaluates it (SSCS_maker.py:154-155). */
int cc_consensus_maker(cc_ctx *ctx, int32_t group_id, double cutoff, int64_t *n_out);
/* re-run read_bam on a resident stream with a new hash seed */
int cc_read_bam_rerun(cc_ctx *ctx, int32_t group_id, uint64_t seed);
/* DCS: duplex pairing + duplex_consensus. bc_swap from ccio_interner_swap_table. */
int cc_duplex_consensus(cc_ctx *ctx, int32_t group_id, const int32_t *bc_swap, int32_t n_bc, int64_t *n_out);
/* Singleton correction against an SSCS group (scope_by_run=1). */
int cc_singleton_correction(cc_ctx *ctx, int32_t singleton_group, int32_t sscs_group, const int32_t *bc_swap,
                            int32_t n_bc, int64_t *n_out);

/* Copy a named result array of a group to host memory; returns bytes copied
 * (or the needed size when dst is NULL).  Names are documented in engine.py. */
int64_t cc_fetch(cc_ctx *ctx, int32_t group_id, const char *name, void *dst, int64_t cap);

/* ---------------------------------------------------------- function-level boundary
 * The reference's per-family functions on caller-given reads.  The reads are
 * records of an uploaded table (cc_table_upload); results are written row by row, out_stride bytes
 * of quality and out_stride/2 bytes of BAM sequence nibbles per row (first base in the high nibble,
 * out_stride even and >= the table's longest read); out_meta[5*k..] = consensus length, mapq,
 * tlen, flag, RG id (-1: none): create_aligned_segment's fields (consensus_helper.py:568-619). */

/* SSCS_maker.consensus_maker(readList, cutoff) (SSCS_maker.py:81-168) for nfam families:
 * family k is the records member_index[fam_offsets[k] .. fam_offsets[k+1]) in readList order
 * (fam_offsets[0] == 0, nfam + 1 entries); the count/pass >= cutoff test in IEEE double.  Returns the
 * CC_E_* of the reference's raise (CC_E_N_HIGHQ, CC_E_BAD_BASE, CC_E_SHORT_READ ...) for any family;
 * CC_E_INVALID for an empty family (readList[0], SSCS_maker.py:107). */
int cc_sscs_vote(cc_ctx *ctx, int32_t table_id, const int32_t *member_index, const int64_t *fam_offsets,
                 int64_t nfam, double cutoff, uint8_t *out_seq_nib, uint8_t *out_qual, int32_t *out_meta,
                 int32_t out_stride);
/* duplex_consensus(read1, read2) for n pairs: read1 = record rec_a[i] of table_a, read2 = rec_b[i] of
 * table_b.  mode 0: DCS_maker.duplex_consensus (DCS_maker.py:99-123; equal bases, min(60, q1+q2));
 * mode 1: singleton_correction.duplex_consensus (singleton_correction.py:61-86; also q1 > 29 and
 * q2 > 29), the record fields then from read1 alone (strand_correction, :89-111). */
int cc_pair_vote(cc_ctx *ctx, int32_t mode, int32_t table_a, int32_t table_b, const int32_t *rec_a,
                 const int32_t *rec_b, int64_t n, uint8_t *out_seq_nib, uint8_t *out_qual, int32_t *out_meta,
                 int32_t out_stride);

/* read_dict / tag_dict grouping (consensus_helper.py:426-500: read_dict[tag].append(read) in input
 * order; families in order of their first read, tag_dict's insertion order) on caller-given keys:
 * n keys of key_bytes bytes each (a multiple of 4, <= 256), compared exactly.  Family k is
 * out_perm[out_fam_offsets[k] .. out_fam_offsets[k+1]) (input indices, increasing); out_fam_offsets
 * holds *out_nfam + 1 entries (capacity n + 1).  The output feeds cc_sscs_vote's member_index /
 * fam_offsets directly.  Replaces SURVEY.md §8b item 3. */
int cc_group(cc_ctx *ctx, int64_t n, const void *keys, int32_t key_bytes, int32_t *out_perm,
             int64_t *out_fam_offsets, int64_t *out_nfam);
/* The duplex pairing on caller-given tags.  Entries i = 0..n-1 are processed
 * in index order (csn_pair_dict order); keys[i] is entry i's tag and partner_keys[i] its duplex_tag
 * (ccio_duplex_tag; any key map works, mutual or not), key_bytes bytes each, compared exactly; the
 * keys of one call are distinct (CC_E_INVALID otherwise).
 *   mode 0, DCS_maker.py:245-282: decision 0 = DCS with entry out_partner[i]; 1 = sscs.singleton
 *     (partner absent); 2 = skipped (the partner made a DCS before: duplex_dict).  CC_E_KEYERROR where
 *     the reference raises (read_dict[ds] deleted: a non-mutual partner processed before).
 *   mode 1, singleton_correction.py:278-319 (entries = singleton tags, x_keys[m] = SSCS tags):
 *     0 = corrected by SSCS x entry out_partner[i] (consumed); 1 = corrected by singleton entry
 *     out_partner[i] (correction_dict bookkeeping); 2 = uncorrected.
 * With out_seq non-NULL the joined pairs are also voted (duplex_consensus, DCS_maker.py:99-123 /
 * singleton_correction.py:61-86 with create_aligned_segment's fields): entry i's read is record
 * rec_a[i] of table_a, SSCS entry k's rec_x[k] of table_x; row i of out_seq / out_qual / out_meta
 * (as cc_pair_vote) holds entry i's consensus when it has one. */
int cc_duplex_join(cc_ctx *ctx, int32_t mode, int64_t n, const void *keys, const void *partner_keys, int64_t m,
                   const void *x_keys, int32_t key_bytes, int32_t *out_decision, int64_t *out_partner,
                   int32_t table_a, const int32_t *rec_a, int32_t table_x, const int32_t *rec_x,
                   uint8_t *out_seq_nib, uint8_t *out_qual, int32_t *out_meta, int32_t out_stride);

/* fastq2bam's UMI extraction decision (extract_barcodes.py:287-405) for n read
 * pairs on the GPU: h1 / h2 hold the first 32 bases of each pair's reads (zero padded, ccio_fq_heads),
 * len1 / len2 the read lengths.  pattern (N = barcode base, A/C/G/T = spacer; <= 32) or the distinct
 * barcode list blist[nblist] (<= 1024 entries of <= 32 bases; the reference's --skipcheck path).
 * Per pair: out_status 0 passing / 1 missing spacer / 2 bad barcode, out_bc (72 bytes per pair: the
 * header barcode 'R1.R2', NUL terminated), out_cut1 / out_cut2 (bases removed), list mode
 * out_bad1 / out_bad2 (ccio_fq_write's masks).  counts[3] = missing spacer, bad barcodes, passing;
 * r1_hist / r2_hist as ccio_extract_barcodes.  CC_E_UNSUPPORTED beyond those sizes (the host path
 * takes them). */
int cc_extract_barcodes(cc_ctx *ctx, int64_t n, const uint8_t *h1, const uint8_t *h2, const int32_t *len1,
                        const int32_t *len2, const char *pattern, const char *const *blist, int32_t nblist,
                        uint8_t *out_status, char *out_bc, int32_t *out_cut1, int32_t *out_cut2, uint32_t *out_bad1,
                        uint32_t *out_bad2, int64_t *counts, int64_t *r1_hist, int64_t *r2_hist);

/* ---------------------------------------------------------- multi-GPU reduction (RCCL over xGMI)
 * The sharded pipeline's one collective.  Rank 0 makes the 128-byte id
 * (cc_comm_unique_id) and hands it to every rank (e.g. torch.distributed broadcast); each rank calls
 * cc_comm_init on its own context's GPU.  RCCL is loaded at run time (dlopen librccl.so.1). */
typedef struct cc_comm cc_comm;
int cc_comm_unique_id(char *id, int32_t cap /* >= 128 */);
int cc_comm_init(cc_ctx *ctx, int32_t world, int32_t rank, const char *id, cc_comm **comm);
int cc_comm_destroy(cc_comm *comm);
/* stats.txt counters and read_families' per-size counts summed, each size's first-seen key
 * (rank << 40 | place) min-reduced, in place; comm NULL (one process): unchanged.  Replaces the
 * reference's per-process counters (SSCS_maker.py:353-408, DCS_maker.py:287-304,
 * singleton_correction.py:324-336) for one sample split over ranks. */
int cc_reduce_stats(cc_ctx *ctx, cc_comm *comm, int64_t *counters, int32_t n_counters, int64_t *fam_count,
                    int64_t *fam_first, int32_t fam_len);
/* v[n] max-reduced in place (the family table's length, per-rank times) */
int cc_allreduce_max(cc_ctx *ctx, cc_comm *comm, int64_t *v, int32_t n);


#ifdef __cplusplus
}
#endif
#endif
