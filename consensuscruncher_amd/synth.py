"""Seeded synthetic UMI-tagged paired-end data (BASELINE.md "Inputs").

Produces a coordinate-sorted batch of BAM records as numpy columns.  It models
what ``ConsensusCruncher.py fastq2bam`` (bwa + samtools sort) would hand to the
consensus stage:

* molecules on one or more contigs, insert ~ N(300, 50);
* barcodes ``b1.b2`` in the qname after ``|`` (extract_barcodes.py:315-318):
  pattern mode ``NNT`` gives 2 random bases per side, list mode draws
  variable-length barcodes from a list (the ``-l`` case, config C5);
* each molecule strand has a PCR family of ``1 + Poisson(fam_mean)`` read pairs
  (or a singleton-heavy law); ``duplex_frac`` of molecules carry both strands,
  the (-) strand with the swapped barcode ``b2.b1`` and flags 83/163 against
  99/147 on the (+) strand (consensus_helper.py:252-305, 639-683);
* 0.5% substitutions, N at Q2, quals 80% Q37 / 10% Q40 / 8% Q25-29 / 2% Q30-36;
* soft clips on ~10% of molecule ends, a few per-read cigar/mapq/RG variants,
  translocated pairs (flags 65/129), and bad reads (unmapped pairs, mate-unmapped
  flags, secondary/supplementary copies, qnames without the delimiter).

Not used by the hot path; used by tests, fixture generation and bench.py.
"""
import numpy as np

BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
SEED_BASE = 20261015


class Batch(object):
    """Columnar records.  Strings are tables + per-record ids."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    @property
    def n(self):
        return len(self.flag)


def _barcode_table(rng, mode, n_list=48):
    if mode == "pattern":
        # NNT: 2 random bases per read end -> 16 half-barcodes
        halves = [a + b for a in "ACGT" for b in "ACGT"]
    else:
        # variable-length barcode list (-l), lengths 3..6
        halves = set()
        while len(halves) < n_list:
            ln = int(rng.integers(3, 7))
            halves.add("".join(rng.choice(list("ACGT"), ln)))
        halves = sorted(halves)
    return halves


def generate(n_pairs, seed=SEED_BASE, read_len=150, contigs=(("chr1", 5_000_000),),
             barcode_mode="pattern", fam_mean=3.0, duplex_frac=0.5, singleton_frac=None,
             clip_frac=0.10, err_rate=0.005, n_rate=0.001, bad_frac=0.01,
             transloc_frac=0.0, loci=None, zipf_s=None, max_fam=5000,
             variant_frac=0.01, spacer_bad_frac=0.002, quirk_frac=0.0, chain_frac=0.0, dupq_frac=0.0,
             shuffle=False, windows=None, mates_anywhere=False, straddle_frac=0.0, pair_offset=0, ties="random"):
    """Generate about ``n_pairs`` read pairs.

    loci: if given (int), molecules start within +-150 bp of that many loci
    (deep targeted-panel case, config C4) with Zipf(``zipf_s``) family sizes.
    singleton_frac: if given, that fraction of strand-families has size 1 and
    the rest sizes 2..6 (config C5).
    barcode_mode "odd": 3-base barcodes without '.', the (-) strand carrying duplex_tag's rotation
    b[1:] + b[:1] of the (+) barcode (consensus_helper.py:663-674), so duplex keys are not mutual;
    chain_frac of the (+) families get a clone family with the twice-rotated barcode (a chain
    t -> duplex(t) -> duplex(duplex(t)) at one locus).
    dupq_frac: that fraction of pairs gets a third record with its qname (the R2 end shifted 1000
    bp), a quarter of them a whole second pair with the qname interleaved 40 bp downstream, and a
    quarter an exact duplicate of both records (pair_dict pairs occurrences in stream order).
    shuffle: records in random order (not coordinate-sorted; read_bam fetches until_eof).
    ties: "random" (default): records at one (tid, pos, strand) in random order; "input": in generation
    order (a stable sort of name-grouped aligner output, as samtools sort leaves it).
    windows: [(tid, start, end)] -- molecules start only inside these intervals (proportional to their
    lengths), translocated mates land in them too: one GPU's block of bed regions of a C3-shaped
    sample (bench.py weak scaling over the cytoband shards).
    mates_anywhere: with windows, translocated mates land anywhere on the contigs (another GPU's block:
    the one sample the ranks of bench.py --gpus N share); straddle_frac: that fraction of molecules
    (windows only) ends past its window, so its right read lies in the next bed region.
    pair_offset: added to every pair id (qnames SYN<id>): disjoint qnames for the ranks' parts.
    quirk_frac: that fraction of pairs gets a clone with flags 67/131 (a second tag with the same
    consensus tag: "Consensus tag NOT UNIQUE", consensus_helper.py:470-487) and a clone whose two
    ends share one tag (flags 1089/1153 at one position: "line read twice", :495-500).
    """
    rng = np.random.default_rng(seed)
    L = int(read_len)
    names = [c[0] for c in contigs]
    lens = np.array([c[1] for c in contigs], dtype=np.int64)
    if barcode_mode == "odd":
        halves = [str(i) for i in range(8)]   # 8 x 8 = 64 ids: the 3-mers
        tri = [a + b + c for a in "ACGT" for b in "ACGT" for c in "ACGT"]
        rot = np.array([tri.index(t[1:] + t[:1]) for t in tri], np.int64)
    else:
        halves = _barcode_table(rng, barcode_mode)
    nh = len(halves)

    # ---- strand-family sizes
    def fam_sizes(k):
        if zipf_s is not None:
            s = rng.zipf(zipf_s, k)
            return np.minimum(s, max_fam).astype(np.int64)
        if singleton_frac is not None:
            s = rng.integers(2, 7, k)
            s[rng.random(k) < singleton_frac] = 1
            return s.astype(np.int64)
        return (1 + rng.poisson(fam_mean, k)).astype(np.int64)

    if zipf_s is not None:   # mean of Zipf(s) clipped at max_fam: sum_{k<M} k p_k + M P(Z >= M)
        zs, M = float(zipf_s), int(max_fam)
        K = 100_000
        kk = np.arange(1, K, dtype=np.float64)
        # zeta(s) and the tail sums by Euler-Maclaurin past K (the draw's support is unbounded)
        zeta = (kk ** -zs).sum() + K ** (1 - zs) / (zs - 1) + 0.5 * K ** -zs
        below = np.arange(1, M, dtype=np.float64)
        p_below = (below ** -zs) / zeta
        fam_avg = float((below * p_below).sum() + M * (1.0 - p_below.sum()))
    elif singleton_frac is not None:
        fam_avg = 1.0 + 3.5 * (1 - singleton_frac)
    else:
        fam_avg = 1.0 + fam_mean
    mean_pairs_per_mol = (1.0 + duplex_frac) * fam_avg
    n_mol = max(1, int(n_pairs / max(mean_pairs_per_mol, 1.0)))

    # ---- molecules
    mol_tid = rng.choice(len(names), n_mol, p=lens / lens.sum()).astype(np.int32)
    ins = np.clip(np.rint(rng.normal(300, 50, n_mol)), L + 10, 3 * L).astype(np.int64)
    if loci is not None:
        loc_tid = rng.choice(len(names), loci, p=lens / lens.sum())
        loc_pos = (rng.random(loci) * (lens[loc_tid] - 4000)).astype(np.int64) + 1000
        which = rng.integers(0, loci, n_mol)
        mol_tid = loc_tid[which].astype(np.int32)
        start = loc_pos[which] + rng.integers(-150, 151, n_mol)
    elif windows is not None:
        win = np.asarray(windows, np.int64).reshape(-1, 3)
        wlen = np.maximum(win[:, 2] - win[:, 1], 1).astype(np.float64)
        wi = rng.choice(len(win), n_mol, p=wlen / wlen.sum())
        mol_tid = win[wi, 0].astype(np.int32)
        start = win[wi, 1] + (rng.random(n_mol) * np.maximum(win[wi, 2] - win[wi, 1] - ins, 1)).astype(np.int64)
        if straddle_frac > 0:   # the right read starts past the window's end (left read inside it)
            we = win[wi, 2]
            sm = (rng.random(n_mol) < straddle_frac) & (we + 2 * ins + 1000 < lens[mol_tid]) & (we - ins > win[wi, 1])
            start[sm] = we[sm] - ins[sm] + L + (rng.random(int(sm.sum())) * (ins[sm] - L)).astype(np.int64)
    else:
        start = (rng.random(n_mol) * np.maximum(lens[mol_tid] - ins - 2000, 1)).astype(np.int64) + 1000
    b1 = rng.integers(0, nh, n_mol)
    b2 = rng.integers(0, nh, n_mol)
    lclip = np.where(rng.random(n_mol) < clip_frac, rng.integers(5, 21, n_mol), 0)
    rclip = np.where(rng.random(n_mol) < clip_frac, rng.integers(5, 21, n_mol), 0)
    transloc = rng.random(n_mol) < transloc_frac if len(names) > 1 else np.zeros(n_mol, bool)
    mate_tid = mol_tid.copy()
    if transloc.any():
        mate_tid[transloc] = (mol_tid[transloc] + rng.integers(1, len(names), transloc.sum())) % len(names)
    right_pos = start + ins - L
    if transloc.any() and windows is not None and not mates_anywhere:
        wj = rng.choice(len(win), int(transloc.sum()), p=wlen / wlen.sum())
        mate_tid[transloc] = win[wj, 0]
        right_pos[transloc] = win[wj, 1] + (rng.random(len(wj)) * wlen[wj]).astype(np.int64)
    elif transloc.any():
        right_pos[transloc] = (rng.random(transloc.sum()) * (lens[mate_tid[transloc]] - 2000)).astype(np.int64) + 1000

    # strands present: 0 -> (+) only, 1 -> (-) only, 2 -> both
    both = rng.random(n_mol) < duplex_frac
    one = rng.integers(0, 2, n_mol)
    has_plus = both | (one == 0)
    has_minus = both | (one == 1)
    fam_plus = np.where(has_plus, fam_sizes(n_mol), 0)
    fam_minus = np.where(has_minus, fam_sizes(n_mol), 0)

    # ---- read pairs: one row per pair
    pm = np.concatenate([np.repeat(np.arange(n_mol), fam_plus), np.repeat(np.arange(n_mol), fam_minus)])
    ps = np.concatenate([np.zeros(fam_plus.sum(), np.int8), np.ones(fam_minus.sum(), np.int8)])
    P = len(pm)
    # left end = lower coordinate end (or the tid-ordered end for translocations)
    # (+): R1 = left (fwd), R2 = right (rev); (-): R1 = right (rev), R2 = left (fwd)
    ltid = mol_tid[pm]
    rtid = mate_tid[pm]
    lpos = start[pm]
    rpos = right_pos[pm]
    ins_p = ins[pm]
    tl = transloc[pm]

    # true sequences per molecule end, then errors per read (sparse draws: fast at 10^7 reads)
    def true_seq(k):
        return BASES[rng.integers(0, 4, (k, L), dtype=np.uint8)]

    mol_left = true_seq(n_mol)
    mol_right = true_seq(n_mol)

    # quality rows drawn from a pool of rows that follow the model
    pool_n = 4096
    u = rng.random((pool_n, L))
    qpool = np.full((pool_n, L), 37, np.uint8)
    qpool[u >= 0.80] = 40
    lowm = (u >= 0.90) & (u < 0.98)
    qpool[lowm] = rng.integers(25, 30, lowm.sum())
    midm = u >= 0.98
    qpool[midm] = rng.integers(30, 37, midm.sum())

    def noisy(truth_rows):
        s = truth_rows.copy()
        k = s.shape[0]
        q = qpool[rng.integers(0, pool_n, k)]
        flat_s = s.reshape(-1)
        flat_q = q.reshape(-1)
        m = rng.binomial(k * L, err_rate)
        if m:
            flat_s[rng.integers(0, k * L, m)] = BASES[rng.integers(0, 4, m)]
        m = rng.binomial(k * L, n_rate)
        if m:
            idx = rng.integers(0, k * L, m)
            flat_s[idx] = ord("N")
            flat_q[idx] = 2
        return s, q

    lseq, lqual = noisy(mol_left[pm])
    rseq, rqual = noisy(mol_right[pm])

    # cigars: table of strings
    cig_table = {}

    def cig_id(s):
        if s not in cig_table:
            cig_table[s] = len(cig_table)
        return cig_table[s]

    lcl = lclip[pm].copy()
    rcl = rclip[pm].copy()
    # a few per-read cigar variants split families (consensus_helper.py:252-305)
    var = rng.random(P) < variant_frac
    lcl[var] = np.where(lcl[var] > 0, 0, 3)
    lcig = np.array([cig_id("%dS%dM" % (c, L - c) if c else "%dM" % L) for c in range(0, 21)])[lcl]
    rcig = np.array([cig_id("%dM%dS" % (L - c, c) if c else "%dM" % L) for c in range(0, 21)])[rcl]

    bc_plus = b1[pm] * nh + b2[pm]
    bc_minus = b2[pm] * nh + b1[pm]
    if barcode_mode == "odd":
        bc_minus = rot[bc_plus]
    bcid = np.where(ps == 0, bc_plus, bc_minus)

    # flags
    l_flag = np.where(ps == 0, 99, 163).astype(np.uint16)
    r_flag = np.where(ps == 0, 147, 83).astype(np.uint16)
    # translocations: no proper-pair, same-direction style flags 65/129 (+) and 129/65 (-)
    l_flag = np.where(tl, np.where(ps == 0, 65, 129), l_flag).astype(np.uint16)
    r_flag = np.where(tl, np.where(ps == 0, 129, 65), r_flag).astype(np.uint16)
    # a few mapq / RG / flag variants inside families (read_mode, consensus_flag ties)
    l_mapq = np.where(rng.random(P) < 0.03, 59, 60).astype(np.uint8)
    r_mapq = np.where(rng.random(P) < 0.03, 59, 60).astype(np.uint8)
    rg = np.where(rng.random(P) < 0.02, 1, 0).astype(np.int32)
    flagvar = (rng.random(P) < 0.01) & ~tl
    l_flag = np.where(flagvar & (ps == 0), 97, l_flag).astype(np.uint16)   # 97: R1 fwd, no proper bit
    r_flag = np.where(flagvar & (ps == 0), 145, r_flag).astype(np.uint16)

    tlen_l = np.where(tl, 0, ins_p).astype(np.int32)
    tlen_r = -tlen_l

    # ---- assemble the two records of every pair
    pair_id = np.arange(P, dtype=np.int64)
    rec = dict(
        pair=np.concatenate([pair_id, pair_id]),
        tid=np.concatenate([ltid, rtid]).astype(np.int32),
        pos=np.concatenate([lpos, rpos]).astype(np.int32),
        mtid=np.concatenate([rtid, ltid]).astype(np.int32),
        mpos=np.concatenate([rpos, lpos]).astype(np.int32),
        tlen=np.concatenate([tlen_l, tlen_r]).astype(np.int32),
        flag=np.concatenate([l_flag, r_flag]).astype(np.uint16),
        mapq=np.concatenate([l_mapq, r_mapq]).astype(np.uint8),
        cig=np.concatenate([lcig, rcig]).astype(np.int32),
        bc=np.concatenate([bcid, bcid]).astype(np.int64),
        rg=np.concatenate([rg, rg]).astype(np.int32),
        srank=np.concatenate([ps, ps]).astype(np.int8),
        seq=np.concatenate([lseq, rseq]),
        qual=np.concatenate([lqual, rqual]),
    )
    spacer_bad = np.zeros(2 * P, bool)

    # ---- bad reads (filters of consensus_helper.py:404-420)
    extra = []
    nb = int(P * bad_frac)
    if nb > 0:
        src = rng.integers(0, 2 * P, nb)
        kind = rng.integers(0, 4, nb)
        for k, flag_or in ((0, 0x100), (1, 0x800)):
            sel = src[kind == k]
            if len(sel):
                d = {key: v[sel].copy() for key, v in rec.items()}
                d["flag"] = (d["flag"] | flag_or).astype(np.uint16)
                d["pair"] = d["pair"]  # same qname as the primary
                extra.append((d, np.zeros(len(sel), bool)))
        # mate-unmapped pairs: mapped read flag 73/137 + unmapped mate placed alongside
        sel = src[kind == 2]
        if len(sel):
            d = {key: v[sel].copy() for key, v in rec.items()}
            d["pair"] = np.arange(len(sel)) + 10 * P + 10
            m = d["flag"].copy()
            d["flag"] = np.where(m & 0x10, 137, 73).astype(np.uint16)   # 137 = 1+8+128, 73 = 1+8+64
            d["mtid"] = d["tid"].copy()
            d["mpos"] = d["pos"].copy()
            d["tlen"][:] = 0
            u = {key: v.copy() for key, v in d.items()}
            u["flag"] = np.where(d["flag"] == 73, 133, 69).astype(np.uint16)  # unmapped mate, placed
            u["mapq"][:] = 0
            u["cig"][:] = -1
            extra.append((d, np.zeros(len(sel), bool)))
            extra.append((u, np.zeros(len(sel), bool)))
        # fully unmapped pairs at the end of the file (tid -1)
        sel = src[kind == 3]
        if len(sel):
            for fl in (77, 141):
                d = {key: v[sel].copy() for key, v in rec.items()}
                d["pair"] = np.arange(len(sel)) + 20 * P + 20
                d["flag"][:] = fl
                d["tid"][:] = -1
                d["pos"][:] = -1
                d["mtid"][:] = -1
                d["mpos"][:] = -1
                d["tlen"][:] = 0
                d["mapq"][:] = 0
                d["cig"][:] = -1
                extra.append((d, np.zeros(len(sel), bool)))
    # qnames without the barcode delimiter (bad spacer)
    nsp = int(P * spacer_bad_frac)
    if nsp:
        spacer_pairs = rng.choice(P, nsp, replace=False)
        spacer_bad[np.isin(rec["pair"], spacer_pairs)] = True
    for d, sb in extra:
        for key in rec:
            rec[key] = np.concatenate([rec[key], d[key]])
        spacer_bad = np.concatenate([spacer_bad, sb])
    if nsp:
        spacer_bad |= np.isin(rec["pair"], spacer_pairs) & (rec["pair"] < P)

    # ---- dictionary quirks of read_bam
    if quirk_frac > 0:
        base_pairs = np.unique(rec["pair"][(rec["flag"] == 99)])
        pick = rng.choice(base_pairs, max(1, int(len(base_pairs) * quirk_frac)), replace=False)
        sel = np.isin(rec["pair"], pick) & ((rec["flag"] == 99) | (rec["flag"] == 147))
        d = {key: v[sel].copy() for key, v in rec.items()}
        d["pair"] = d["pair"] + 30 * P + 30
        d["flag"] = np.where(d["flag"] == 99, 67, 131).astype(np.uint16)     # both forward, proper
        extra_q = [(d, np.zeros(sel.sum(), bool))]
        left = (rec["flag"] == 99) & np.isin(rec["pair"], pick[: max(1, len(pick) // 2)])
        for fl in (1089, 1153):                                                # dup-flag pair, one position
            d = {key: v[left].copy() for key, v in rec.items()}
            d["pair"] = d["pair"] + 40 * P + 40
            d["flag"][:] = fl
            d["mtid"] = d["tid"].copy()
            d["mpos"] = d["pos"].copy()
            d["tlen"][:] = 0
            extra_q.append((d, np.zeros(left.sum(), bool)))
        for d, sb in extra_q:
            for key in rec:
                rec[key] = np.concatenate([rec[key], d[key]])
            spacer_bad = np.concatenate([spacer_bad, sb])

    # ---- non-mutual duplex chains: a clone of a (+) family with the twice-rotated barcode
    if chain_frac > 0 and barcode_mode == "odd":
        lead = (rec["flag"] == 99) & (rec["pair"] < P)
        fkey = rec["tid"][lead].astype(np.int64) * (1 << 40) + rec["pos"][lead].astype(np.int64) * 64 + rec["bc"][lead]
        ukeys = np.unique(fkey)
        pick = rng.choice(ukeys, max(1, int(len(ukeys) * chain_frac)), replace=False)
        pairs = np.unique(rec["pair"][lead][np.isin(fkey, pick)])
        sel = np.isin(rec["pair"], pairs)
        d = {key: v[sel].copy() for key, v in rec.items()}
        d["pair"] = d["pair"] + 50 * P + 50
        d["bc"] = rot[rot[d["bc"]]]
        d["srank"][:] = 2
        sb = spacer_bad[sel]
        for key in rec:
            rec[key] = np.concatenate([rec[key], d[key]])
        spacer_bad = np.concatenate([spacer_bad, sb])
    # ---- qnames seen more than twice (pair_dict pairs occurrences in stream order)
    if dupq_frac > 0:
        prim = np.unique(rec["pair"][(rec["flag"] == 99) & (rec["pair"] < P)])
        pick = rng.choice(prim, max(4, int(len(prim) * dupq_frac)), replace=False)
        q = len(pick) // 4
        third, inter, dup = pick[2 * q:], pick[:q], pick[q:2 * q]
        add = []
        sel = np.isin(rec["pair"], third) & (rec["flag"] == 147)
        d = {key: v[sel].copy() for key, v in rec.items()}
        d["pos"] = d["pos"] + 1000
        add.append((d, spacer_bad[sel]))
        sel = np.isin(rec["pair"], inter) & ((rec["flag"] == 99) | (rec["flag"] == 147))
        d = {key: v[sel].copy() for key, v in rec.items()}
        d["pos"] = d["pos"] + 40
        d["mpos"] = d["mpos"] + 40
        add.append((d, spacer_bad[sel]))
        sel = np.isin(rec["pair"], dup) & ((rec["flag"] == 99) | (rec["flag"] == 147))
        add.append(({key: v[sel].copy() for key, v in rec.items()}, spacer_bad[sel]))
        for d, sb in add:
            for key in rec:
                rec[key] = np.concatenate([rec[key], d[key]])
            spacer_bad = np.concatenate([spacer_bad, sb])

    if pair_offset:
        rec["pair"] = rec["pair"].astype(np.int64) + int(pair_offset)

    # ---- coordinate sort (samtools key, random tie order)
    tkey = rec["tid"].astype(np.int64)
    tkey[tkey < 0] = 1 << 40
    rev = (rec["flag"] & 0x10) > 0
    tie = rng.permutation(len(tkey)) if ties == "random" else np.arange(len(tkey))
    if barcode_mode == "odd":
        # ties: (+) strand records, then (-), then chain clones, so that the reference's DCS stage
        # meets every duplex chain head first (the other orders end in its KeyError, DCS_maker.py:258)
        tie = rec["srank"].astype(np.int64) * len(tkey) + tie
    order = np.lexsort((tie, rev, rec["pos"].astype(np.int64) + 1, tkey))
    if shuffle:
        order = rng.permutation(len(tkey))
    for key in rec:
        rec[key] = rec[key][order]
    spacer_bad = spacer_bad[order]

    cig_strings = [None] * len(cig_table)
    for s, i in cig_table.items():
        cig_strings[i] = s
    if barcode_mode == "odd":
        bc_strings = tri
    else:
        bc_strings = [halves[i // nh] + "." + halves[i % nh] for i in range(nh * nh)]
    return Batch(names=names, lens=[int(x) for x in lens], read_len=L,
                 cigar_table=cig_strings, barcode_table=bc_strings, rg_table=["1", "2"],
                 spacer_bad=spacer_bad, **rec)


def _read_tagged_fastq(path):
    """(ids, barcodes, seqs, quals) of a barcode-extracted FASTQ (extract_barcodes.py:315-318 headers
    '@<id>|<R1 bc>.<R2 bc>/<1|2>')."""
    ids, bcs, seqs, quals = [], [], [], []
    with open(path) as f:
        while True:
            h = f.readline()
            if not h:
                break
            sq = f.readline().rstrip("\r\n")
            f.readline()
            ql = f.readline().rstrip("\r\n")
            name = h[1:].rstrip().rsplit("/", 1)[0]
            i, bc = name.split("|", 1)
            ids.append(i)
            bcs.append(bc)
            seqs.append(sq)
            quals.append(ql)
    return ids, bcs, seqs, quals


_COMP = bytes.maketrans(b"ACGTN", b"TGCAN")


def fastq_surrogate(r1_fastq, r2_fastq, contig=("chr1", 2_000_000), key_len=20, seed=SEED_BASE + 1):
    """C1 surrogate: the bundled test FASTQ pairs, barcodes extracted per NNT, placed at
    coordinates derived from their own sequence instead of a bwa alignment (no aligner or genome here).
    A pair's molecule key is its two read starts (first key_len bases of R1 and R2) in canonical order,
    so PCR copies of one strand share a position (a family) and the other strand, whose R1 starts where
    this strand's R2 does and whose barcode halves are swapped, lands on the same key in the mirrored
    orientation (a duplex partner).  The key's hash gives the position and an insert of 200-399 bp; the
    pair is written as a proper pair (99/147 when R1's start is the smaller, else 163/83), reverse reads
    reverse-complemented, cigar <len>M, mapq 60, RG 1.  Qnames are '<fastq id>|<R1 bc>.<R2 bc>' (bwa
    drops the /1 /2).  Returns a coordinate-sorted Batch."""
    import zlib
    ids1, bcs, s1, q1 = _read_tagged_fastq(r1_fastq)
    ids2, _, s2, q2 = _read_tagged_fastq(r2_fastq)
    if ids1 != ids2:
        raise ValueError("R1 and R2 ids differ")
    L = len(s1[0]) if s1 else 0
    if any(len(x) != L for x in s1 + s2):
        raise ValueError("the surrogate expects one read length")
    P = len(ids1)
    span = contig[1] - 1000
    pos_l = np.zeros(P, np.int64)
    ins = np.zeros(P, np.int64)
    top = np.zeros(P, bool)
    for k in range(P):
        a, b = s1[k][:key_len], s2[k][:key_len]
        top[k] = a <= b
        key = (a + "/" + b) if top[k] else (b + "/" + a)
        h = zlib.crc32(key.encode(), seed & 0xffffffff)
        pos_l[k] = h % span
        ins[k] = 200 + (zlib.crc32(key.encode(), (seed + 1) & 0xffffffff) % 200)
    pos_r = pos_l + ins - L

    def fwd(x):
        return np.frombuffer(x.encode(), np.uint8)

    def rev(x, q):
        return np.frombuffer(x.encode().translate(_COMP)[::-1], np.uint8), np.frombuffer(q.encode()[::-1], np.uint8)

    seq = np.zeros((2 * P, L), np.uint8)
    qual = np.zeros((2 * P, L), np.uint8)
    pos = np.zeros(2 * P, np.int64)
    mpos = np.zeros(2 * P, np.int64)
    flag = np.zeros(2 * P, np.uint16)
    tlen = np.zeros(2 * P, np.int32)
    for k in range(P):
        if top[k]:   # R1 forward at the left end, R2 reverse at the right end
            seq[k], qual[k] = fwd(s1[k]), fwd(q1[k]) - 33
            rs, rq = rev(s2[k], q2[k])
            seq[P + k], qual[P + k] = rs, rq - 33
            pos[k], pos[P + k] = pos_l[k], pos_r[k]
            flag[k], flag[P + k] = 99, 147
            tlen[k], tlen[P + k] = ins[k], -ins[k]
        else:        # R2 forward at the left end, R1 reverse at the right end
            rs, rq = rev(s1[k], q1[k])
            seq[k], qual[k] = rs, rq - 33
            seq[P + k], qual[P + k] = fwd(s2[k]), fwd(q2[k]) - 33
            pos[k], pos[P + k] = pos_r[k], pos_l[k]
            flag[k], flag[P + k] = 83, 163
            tlen[k], tlen[P + k] = -ins[k], ins[k]
        mpos[k], mpos[P + k] = pos[P + k], pos[k]
    bc_table = list(dict.fromkeys(bcs))
    bid = {b: i for i, b in enumerate(bc_table)}
    pair = np.concatenate([np.arange(P), np.arange(P)]).astype(np.int64)
    rec = dict(pair=pair, tid=np.zeros(2 * P, np.int32), pos=pos.astype(np.int32), mtid=np.zeros(2 * P, np.int32),
               mpos=mpos.astype(np.int32), tlen=tlen, flag=flag, mapq=np.full(2 * P, 60, np.uint8),
               cig=np.zeros(2 * P, np.int32), bc=np.array([bid[b] for b in bcs] * 2, np.int64),
               rg=np.zeros(2 * P, np.int32), srank=np.zeros(2 * P, np.int8), seq=seq, qual=qual)
    order = np.lexsort((np.arange(2 * P), (rec["flag"] & 0x10) > 0, rec["pos"].astype(np.int64)))
    for key in rec:
        rec[key] = rec[key][order]
    return Batch(names=[contig[0]], lens=[int(contig[1])], read_len=L, cigar_table=["%dM" % L],
                 barcode_table=bc_table, rg_table=["1", "2"], spacer_bad=np.zeros(2 * P, bool),
                 qnames=[ids1[k] for k in rec["pair"]], **rec)


def qname_of(batch, i, delim="|"):
    if getattr(batch, "qnames", None) is not None:   # fastq_surrogate: real ids
        return "%s%s%s" % (batch.qnames[i], delim, batch.barcode_table[int(batch.bc[i])])
    p = int(batch.pair[i])
    if batch.spacer_bad[i]:
        return "SYN%010d" % p
    return "SYN%010d%s%s" % (p, delim, batch.barcode_table[int(batch.bc[i])])


def sam_header_text(batch):
    lines = ["@HD\tVN:1.6\tSO:coordinate"]
    for n, ln in zip(batch.names, batch.lens):
        lines.append("@SQ\tSN:%s\tLN:%d" % (n, ln))
    lines.append("@RG\tID:1\tSM:synthetic")
    lines.append("@RG\tID:2\tSM:synthetic")
    return "\n".join(lines) + "\n"


def qname_blob(batch, delim="|"):
    """(uint8 blob, int64 offsets[n+1]) of all qnames, vectorized (1-char delimiter)."""
    n = batch.n
    if getattr(batch, "qnames", None) is not None:
        names = [qname_of(batch, i, delim).encode() for i in range(n)]
        off = np.zeros(n + 1, np.int64)
        np.cumsum([len(x) for x in names], out=off[1:])
        return np.frombuffer(b"".join(names), np.uint8).copy(), off
    pair = batch.pair.astype(np.int64)
    digits = np.zeros((n, 10), np.uint8)
    x = pair.copy()
    for k in range(9, -1, -1):
        digits[:, k] = 48 + (x % 10)
        x //= 10
    bct = [s.encode() for s in batch.barcode_table]
    bclen = np.array([len(s) for s in bct], np.int64)
    this_len = np.where(batch.spacer_bad, 0, 1 + bclen[batch.bc])
    lens = 13 + this_len
    off = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    blob = np.zeros(int(off[-1]), np.uint8)
    base = off[:-1]
    blob[base[:, None] + np.arange(3)] = np.frombuffer(b"SYN", np.uint8)
    blob[base[:, None] + 3 + np.arange(10)] = digits
    good = ~batch.spacer_bad
    blob[base[good] + 13] = ord(delim)
    maxbc = int(bclen.max())
    bcmat = np.zeros((len(bct), maxbc), np.uint8)
    for i, s in enumerate(bct):
        bcmat[i, :len(s)] = np.frombuffer(s, np.uint8)
    gi = np.nonzero(good)[0]
    for j in range(maxbc):
        sel = gi[bclen[batch.bc[gi]] > j]
        blob[base[sel] + 14 + j] = bcmat[batch.bc[sel], j]
    return blob, off


CONFIGS = {
    # C1 surrogate: small, 126 bp reads (bundled FASTQ length), hg19-like single contig
    "c1": dict(n_pairs=10_000, read_len=126, contigs=(("chr1", 2_000_000),), fam_mean=0.3),
    # C2: 10 M pairs 2x150, NNT barcodes, mean family size 4, one contig, -b False
    "c2": dict(n_pairs=10_000_000, read_len=150, contigs=(("chr1", 100_000_000),), fam_mean=3.0),
    # C3: 200 M pairs over hg38 (the bundled hg38_cytoBand.txt contigs at their lengths, 0.1%
    # translocations), split over the GPUs by cytoband blocks; n_pairs is per GPU (bench.py weak
    # scaling: each rank generates its block's share, see c3_windows)
    "c3": dict(n_pairs=10_000_000, read_len=150, contigs="hg38_cytoBand.txt", transloc_frac=0.001, bed=True),
    # C4: deep targeted panel, Zipf family sizes up to 5000
    "c4": dict(n_pairs=25_000_000, read_len=150, contigs=(("chr1", 50_000_000),), loci=100,
               zipf_s=1.2, max_fam=5000),
    # C5: singleton-heavy, barcode list with variable lengths
    "c5": dict(n_pairs=1_000_000, read_len=150, contigs=(("chr1", 20_000_000),),
               barcode_mode="list", singleton_frac=0.7, fam_mean=3.0),
}


DATA = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "data")


def band_contigs(name):
    """(contig, length) of a bundled cytoband table, in its order of first appearance."""
    import os
    ends = {}
    for line in open(os.path.join(DATA, name)):
        c = line.split("\t")
        ends[c[0]] = max(ends.get(c[0], 0), int(c[2]))
    return tuple(ends.items())


def c3_windows(world, rank, bed="hg38_cytoBand.txt"):
    """(contigs, windows, bedfile) of rank's block of the cytoband regions: blocks of consecutive bed
    regions (bed order) with near-equal bp, i.e. near-equal reads at uniform coverage (shard.plan_blocks)."""
    import os
    from .consensus_helper import region_list
    from .shard import plan_blocks
    path = os.path.join(DATA, bed)
    contigs = band_contigs(bed)
    tid = {n: i for i, (n, _) in enumerate(contigs)}
    regions = region_list(path)
    lo, hi = plan_blocks([max(e - s, 0) for _, _, s, e in regions], world)[rank]
    win = [(tid[c], s, e) for _, c, s, e in regions[lo:hi] if e > s]
    return contigs, win, path


def config(name, world=1, rank=0):
    """generate() keyword arguments of a CONFIGS entry (c3: rank's block of the cytoband regions) and the
    bed file it runs with (None: -b False)."""
    cfg = dict(CONFIGS[name])
    bed = None
    if cfg.pop("bed", False):
        contigs, win, bed = c3_windows(world, rank, cfg["contigs"])
        cfg["contigs"], cfg["windows"] = contigs, win
    return cfg, bed


_CIG_OPS = {c: i for i, c in enumerate("MIDNSHP=XB")}


def _encode_cigar(s):
    out, num = [], ""
    for ch in s:
        if ch.isdigit():
            num += ch
        else:
            out.append((int(num) << 4) | _CIG_OPS[ch])
            num = ""
    return out


def write_bam_native(batch, path, level=1, delim="|", nthreads=0):
    """Write a Batch through libccio's columnar writer (fast path for large inputs)."""
    import ctypes as C
    from . import native as N
    qn, qoff = qname_blob(batch, delim)
    ops, coff = [], [0]
    for s in batch.cigar_table:
        e = _encode_cigar(s)
        ops.extend(e)
        coff.append(len(ops))
    ops = np.array(ops if ops else [0], np.uint32)
    coff = np.array(coff, np.int64)
    names = (C.c_char_p * len(batch.names))(*[x.encode() for x in batch.names])
    lens = np.array(batch.lens, np.int32)
    rgv = (C.c_char_p * len(batch.rg_table))(*[x.encode() for x in batch.rg_table])
    seq = np.ascontiguousarray(batch.seq, np.uint8)
    qual = np.ascontiguousarray(batch.qual, np.uint8)
    cols = [np.ascontiguousarray(getattr(batch, f), dt) for f, dt in
            (("tid", np.int32), ("pos", np.int32), ("mtid", np.int32), ("mpos", np.int32), ("tlen", np.int32),
             ("flag", np.uint16), ("mapq", np.uint8))]
    cig = np.ascontiguousarray(batch.cig, np.int32)
    rg = np.ascontiguousarray(batch.rg, np.int32)
    rc = N.io().ccio_write_columns(path.encode(), sam_header_text(batch).encode(), len(batch.names),
                                   C.cast(names, N.P), N.ptr(lens), batch.n, *[N.ptr(c) for c in cols],
                                   N.ptr(qn), N.ptr(qoff), N.ptr(cig), N.ptr(ops), N.ptr(coff), batch.read_len,
                                   N.ptr(seq), N.ptr(qual), N.ptr(rg), C.cast(rgv, N.P), level, nthreads)
    if rc != 0:
        raise IOError(N.io_error())
    return path
