"""CPU oracle: a clean-room restatement of ConsensusCruncher's consensus mode.

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product.  It works on records read
through the pysam shim (oracle/shim) and writes BAMs through it.

Pinned against the reference: tests/test_oracle_golden.py runs this module on
every case of tests/golden (outputs of the unmodified reference scripts, see
oracle/make_golden.py) and requires identical records, stats and family tables.

Semantics restated (file:line of the reference each piece follows):
  read_number         consensus_helper.py:57-81
  strand_of           consensus_helper.py:84-156
  ordered_cigars      consensus_helper.py:159-196
  molecule_name       consensus_helper.py:199-249   (sscs_qname)
  read_end_key        consensus_helper.py:252-305   (unique_tag)
  FamilyBuilder.feed  consensus_helper.py:308-506   (read_bam)
  most_common_first / pick_flag / new_record   consensus_helper.py:509-619
  complement_key      consensus_helper.py:639-683   (duplex_tag)
  single_strand_vote  SSCS_maker.py:81-168          (consensus_maker)
  pair_vote           DCS_maker.py:99-123, singleton_correction.py:61-86
  duplex_name         DCS_maker.py:60-96            (dcs_consensus_tag)
  sscs_stage          SSCS_maker.py:183-425
  dcs_stage           DCS_maker.py:130-317
  sc_stage            singleton_correction.py:118-345
  consensus_pipeline  ConsensusCruncher.py:127-346
Mode ties pick the first-seen value (the reference draws randint(0, k-1); the
fixtures patch it to 0).
"""
import collections
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for _p in (HERE, os.path.join(HERE, "shim")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import pysam  # noqa: E402  (shim)
from samtools_shim import samtools_merge, samtools_sort_index  # noqa: E402

FIRST_OF_PAIR = frozenset((99, 83, 67, 115, 81, 97, 65, 113))
SECOND_OF_PAIR = frozenset((147, 163, 131, 179, 161, 145, 129, 177))
STRAND_POS = frozenset((99, 147, 67, 131))
STRAND_NEG = frozenset((83, 163, 115, 179))
STRAND_BY_COORD = frozenset((65, 129, 113, 177, 81, 161, 97, 145))
MATE_UNMAPPED = frozenset((73, 89, 121, 153, 185, 137))
BASE_ORDER = "ACGTN"


class OracleError(Exception):
    """Raised where the reference raises (IndexError / ValueError / KeyError ...)."""


# ------------------------------------------------------------------ keys
def read_number(flag):
    if flag in FIRST_OF_PAIR:
        return "R1"
    if flag in SECOND_OF_PAIR:
        return "R2"
    return None


def strand_of(r):
    f = r.flag
    if f in STRAND_POS:
        return "pos"
    if f in STRAND_NEG:
        return "neg"
    if f in STRAND_BY_COORD:
        num = read_number(f)
        a, b = r.reference_id, r.next_reference_id
        x, y = r.reference_start, r.next_reference_start
        if a != b:
            lower_first = a < b
        else:
            lower_first = x < y if num == "R1" else None
        if num == "R1":
            return "pos" if (a < b or (a == b and x < y)) else "neg"
        return "pos" if (a > b or (a == b and x > y)) else "neg"
    return None


def ordered_cigars(first, second):
    s, num = strand_of(first), read_number(first.flag)
    own_first = (s == "pos" and num == "R1") or (s == "neg" and num == "R2")
    a, b = (first, second) if own_first else (second, first)
    return "%s_%s" % (a.cigarstring, b.cigarstring)


def molecule_name(first, second, barcode, cigars):
    c1, p1 = first.reference_id, first.reference_start
    c2, p2 = second.reference_id, second.reference_start
    if c1 > c2 or (c1 == c2 and p1 > p2):
        c1, p1, c2, p2 = c2, p2, c1, p1
    return "_".join(str(x) for x in (barcode, c1, p1, c2, p2, cigars, strand_of(first),
                                      abs(first.template_length)))


def read_end_key(r, barcode, cigars):
    return "_".join(str(x) for x in (barcode, r.reference_id, r.reference_start, r.next_reference_id,
                                      r.next_reference_start, cigars, "rev" if r.is_reverse else "fwd",
                                      read_number(r.flag)))


def complement_key(key):
    parts = key.split("_")
    bc = parts[0]
    if "." in bc:
        k = bc.index(".")
        parts[0] = bc[k + 1:] + "." + bc[:k]
    else:
        h = len(bc) // 2
        parts[0] = bc[h:] + bc[:h]
    parts[8] = "R2" if parts[8] == "R1" else "R1"
    return "_".join(parts)


# ------------------------------------------------------------------ family building
class FamilyBuilder(object):
    """State of read_bam across regions: pending mates, families, entries."""

    def __init__(self):
        self.pending = collections.defaultdict(list)   # qname -> records (pair_dict)
        self.members = collections.OrderedDict()       # read-end key -> records (read_dict)
        self.size = collections.defaultdict(int)       # read-end key -> count (tag_dict)
        self.entries = collections.defaultdict(list)   # molecule name -> keys (csn_pair_dict)

    def feed(self, records, region=None, delim=None, duplex=False, bad_sink=None):
        n_total = n_unmapped = n_mate = n_multi = n_spacer = 0
        for r in records:
            if region is not None and (r.reference_start < region[0] or r.reference_start > region[1]):
                continue
            n_total += 1
            kind = "ok"
            if delim is not None and delim not in r.query_name:
                kind, n_spacer = "spacer", n_spacer + 1
            elif r.is_unmapped:
                kind, n_unmapped, n_total = "unmapped", n_unmapped + 1, n_total - 1
            elif r.flag in MATE_UNMAPPED:
                kind, n_mate = "mate", n_mate + 1
            elif r.is_secondary or r.is_supplementary:
                kind, n_multi = "multi", n_multi + 1
            if kind != "ok" and bad_sink is not None:
                bad_sink.append(r)
                continue
            waiting = self.pending[r.query_name]
            waiting.append(r)
            if len(waiting) < 2:
                continue
            first, second = waiting[0], waiting[1]
            if duplex:
                barcode = first.query_name.split("_")[0]
            else:
                barcode = first.query_name.split(delim if delim is not None else "|")[1]
            cig = ordered_cigars(first, second)
            mol = molecule_name(first, second, barcode, cig)
            for rec in (first, second):
                key = read_end_key(rec, barcode, cig)
                if key not in self.members and key not in self.size:
                    self.members[key] = [rec]
                    self.size[key] += 1
                    ent = self.entries[mol]
                    if len(ent) < 2:
                        ent.append(key)          # else: "Consensus tag NOT UNIQUE" (orphan key)
                elif key in self.size and key not in self.members:
                    # read_dict[tag] of a family emitted in an earlier region (overlapping bed regions)
                    raise OracleError("KeyError: %s (consensus_helper.py:490)" % key)
                elif key in self.size and first not in self.members[key]:
                    self.members[key].append(rec)
                    self.size[key] += 1
                # else: "line read twice" -- record dropped
            del self.pending[r.query_name]
        return n_total, n_mate, n_multi, n_spacer


def most_common_first(values):
    counts = collections.Counter(values)
    top = max(counts.values())
    for v in counts:                 # Counter keeps first-seen order
        if counts[v] == top:
            return v


def pick_flag(records):
    counts = collections.Counter(r.flag for r in records)
    top = max(counts.values())
    best = [f for f in counts if counts[f] == top]
    if len(best) == 1:
        return best[0]
    for f in (99, 83, 147, 163):
        if f in best:
            return f
    return best[0]


def new_record(members, seq, quals, name):
    t = members[0]
    r = pysam.AlignedSegment(t.header)
    r.query_name = name
    r.query_sequence = seq
    r.reference_id = t.reference_id
    r.reference_start = t.reference_start
    r.mapping_quality = most_common_first([m.mapping_quality for m in members])
    r.cigar = t.cigar
    r.next_reference_id = t.next_reference_id
    r.next_reference_start = t.next_reference_start
    r.template_length = most_common_first([m.template_length for m in members])
    r.query_qualities = quals
    r.flag = pick_flag(members)
    try:
        r.set_tag("RG", most_common_first([m.get_tag("RG") for m in members]))
    except KeyError:
        pass
    return r


# ------------------------------------------------------------------ votes
def single_strand_vote(members, cutoff):
    L = members[0].infer_query_length()
    if L is None:
        raise OracleError("TypeError: no cigar")
    n = len(members)
    seqs = [m.query_sequence for m in members]
    quals = [m.query_qualities for m in members]
    out_s, out_q = [], []
    for i in range(L):
        cnt = [0, 0, 0, 0, 0]
        qsum = [0, 0, 0, 0, 0]
        failed = 0
        for s, q in zip(seqs, quals):
            if q is None:
                raise OracleError("TypeError: qualities missing")
            if i >= len(q) or i >= len(s):
                raise OracleError("IndexError: read shorter than consensus")
            b = BASE_ORDER.find(s[i])
            if b < 0:
                raise OracleError("ValueError: base %r" % s[i])
            if q[i] < 30:
                failed += 1
            else:
                if b == 4:
                    raise OracleError("IndexError: N with quality >= 30")
                cnt[b] += 1
                qsum[b] += q[i]
        top = max(cnt)
        k = cnt.index(top)
        mq = min(60, qsum[k])
        passed = n - failed
        if passed and cnt[k] / passed >= cutoff:
            out_s.append(BASE_ORDER[k])
        else:
            out_s.append("N")
        out_q.append(mq)
    return "".join(out_s), out_q


def pair_vote(a, b, gate):
    sa, sb = a.query_sequence or "", b.query_sequence or ""
    qa, qb = a.query_qualities, b.query_qualities
    out_s, out_q = [], []
    for i in range(a.query_length):
        if i >= len(sb):
            raise OracleError("IndexError: complement shorter")
        same = sa[i] == sb[i]
        if same and (gate or True):
            if qa is None or qb is None:
                raise OracleError("TypeError: qualities missing")
        if same and (not gate or (qa[i] > 29 and qb[i] > 29)):
            out_s.append(sa[i])
            out_q.append(min(60, qa[i] + qb[i]))
        else:
            out_s.append("N")
            out_q.append(0)
    return "".join(out_s), out_q


def duplex_name(tag_name, ds_name):
    bc, dbc = tag_name.split("_")[0], ds_name.split("_")[0]
    coords = tag_name.split("_", 1)[1].rsplit("_", 1)[0]
    n_tag, n_ds = tag_name.split(":")[1], ds_name.split(":")[1]
    if "pos" in tag_name:
        return "%s_%s_%s:%s_%s" % (bc, dbc, coords, n_tag, n_ds)
    return "%s_%s_%s:%s_%s" % (dbc, bc, coords, n_ds, n_tag)


# ------------------------------------------------------------------ function-level joins
def group_keys(keys):
    """read_dict[tag].append(i) over keys in input order (consensus_helper.py:455-500): the families
    in tag_dict insertion order, members in input order (cc_group's contract)."""
    fams = collections.OrderedDict()
    for i, k in enumerate(keys):
        fams.setdefault(k, []).append(i)
    return list(fams.values())


def dcs_join(keys, partners):
    """DCS_maker.py:245-282's per-tag loop over keys in processing order (partners[i] =
    duplex_tag(keys[i])): decision 0 DCS with entry j, 1 sscs.singleton, 2 skipped; raises where the
    reference's read_dict[ds] raises KeyError."""
    index = {k: i for i, k in enumerate(keys)}   # tag_dict (every entry's tag)
    live = set(keys)                              # read_dict
    used = set()                                  # duplex_dict
    out = []
    for i, k in enumerate(keys):
        ds = partners[i]
        if ds in used:
            out.append((2, -1))
            continue
        if ds in index:
            if ds not in live:
                raise OracleError("KeyError: %r (DCS_maker.py:258)" % (ds,))
            out.append((0, index[ds]))
            used.add(k)
        else:
            out.append((1, -1))
        live.discard(k)
    return out


def sc_join(keys, partners, sscs_keys):
    """singleton_correction.py:278-319's per-tag loop (partners[i] = duplex_tag(keys[i])): 0 corrected
    by SSCS entry j (deleted from sscs_dict), 1 corrected by singleton entry j (correction_dict), 2
    uncorrected."""
    sidx = {k: i for i, k in enumerate(sscs_keys)}
    sscs_live = set(sscs_keys)                    # sscs_dict
    index = {k: i for i, k in enumerate(keys)}
    live = set(keys)                              # singleton_dict
    corr = {}                                     # correction_dict
    out = []
    for i, k in enumerate(keys):
        ds = partners[i]
        if ds in sscs_live:
            out.append((0, sidx[ds]))
            sscs_live.discard(ds)
            live.discard(k)
        elif ds in live:
            out.append((1, index[ds]))
            corr[k] = ds
            if ds in corr:
                for x in (k, ds):
                    if x not in live:
                        raise OracleError("KeyError: %r (singleton_correction.py:302)" % (x,))
                    live.discard(x)
                for x in (k, ds):
                    if x not in corr:
                        raise OracleError("KeyError: %r (singleton_correction.py:304)" % (x,))
                    del corr[x]
        else:
            out.append((2, -1))
            live.discard(k)
    return out


# ------------------------------------------------------------------ regions
def regions_of(bedfile):
    if bedfile is None:
        return [(None, None, None, None)]
    table = collections.OrderedDict()
    for line in open(bedfile):
        col = line.split("\t")
        table["%s_%s" % (col[0], col[3])] = (int(col[1]), int(col[2]))
    return [(k, k.rsplit("_", 1)[0], v[0], v[1]) for k, v in table.items()]


def fetch(bam, chrom, start, end):
    if chrom is None:
        return bam.fetch(until_eof=True)
    return bam.fetch(chrom, start, end)


# ------------------------------------------------------------------ stages
def sscs_stage(infile, outfile, cutoff, bedfile=None, bdelim="|"):
    bam = pysam.AlignmentFile(infile, "rb")
    prefix = outfile.split(".sscs")[0]
    sscs_out, single_out, bad = [], [], []
    fb = FamilyBuilder()
    totals = [0, 0, 0, 0]
    for key, chrom, start, end in regions_of(bedfile):
        got = fb.feed(fetch(bam, chrom, start, end), None if chrom is None else (start, end), delim=bdelim,
                      duplex=False, bad_sink=bad)
        totals = [a + b for a, b in zip(totals, got)]
        for mol in list(fb.entries):
            keys = fb.entries[mol]
            if len(keys) != 2:
                continue
            for k in keys:
                fam = fb.members[k]
                name = "%s:%d" % (mol, fb.size[k])
                if fb.size[k] == 1:
                    fam[0].query_name = name
                    single_out.append(fam[0])
                else:
                    seq, q = single_strand_vote(fam, float(cutoff))
                    sscs_out.append(new_record(fam, seq, q, name))
                del fb.members[k]
            del fb.entries[mol]
    for path, recs in ((outfile, sscs_out), ("%s.singleton.bam" % prefix, single_out),
                       ("%s.badReads.bam" % prefix, bad)):
        w = pysam.AlignmentFile(path, "wb", template=bam)
        for r in recs:
            w.write(r)
        w.close()
    stats = ("# === SSCS ===\nUncollapsed - Total reads: {}\nUncollapsed - Unmapped reads: {}\n"
             "Uncollapsed - Secondary/Supplementary reads: {}\nSSCS reads: {}\nSingletons: {}\n"
             "Bad spacers: {}\n").format(totals[0], totals[1], totals[2], len(sscs_out), len(single_out), totals[3])
    with open("%s.stats.txt" % prefix, "w") as f:
        f.write(stats)
    freq = collections.Counter(fb.size.values())
    with open(prefix + ".read_families.txt", "w") as f:
        f.write("family_size\tfrequency\n")
        f.write("\n".join("%s\t%s" % kv for kv in freq.items()))
    if not freq:
        raise OracleError("IndexError: empty family table (SSCS_maker.py:417)")
    return dict(sscs=len(sscs_out), singletons=len(single_out))


def dcs_stage(infile, outfile, bedfile=None):
    bam = pysam.AlignmentFile(infile, "rb")
    if ".dcs.sc" in outfile:
        single_path = "%s.sscs.sc.singleton.bam" % outfile.split(".dcs.sc")[0]
        title, sc = "DCS - Singleton Correction", " SC"
    else:
        single_path = "%s.sscs.singleton.bam" % outfile.split(".dcs")[0]
        title, sc = "DCS", ""
    prefix = outfile.split(".dcs")[0]
    fb = FamilyBuilder()
    used = set()
    dcs_out, single_out = [], []
    totals = [0, 0, 0, 0]
    for key, chrom, start, end in regions_of(bedfile):
        got = fb.feed(fetch(bam, chrom, start, end), None if chrom is None else (start, end), duplex=True)
        totals = [a + b for a, b in zip(totals, got)]
        for mol in list(fb.entries):
            for k in fb.entries[mol]:
                partner = complement_key(k)
                if partner not in used:
                    if k in fb.size and partner in fb.size:
                        if partner not in fb.members:
                            raise OracleError("KeyError: %s" % partner)
                        a, b = fb.members[k][0], fb.members[partner][0]
                        seq, q = pair_vote(a, b, gate=False)
                        dcs_out.append(new_record([a, b], seq, q, duplex_name(a.query_name, b.query_name)))
                        used.add(k)
                    else:
                        single_out.append(fb.members[k][0])
                    del fb.members[k]
            del fb.entries[mol]
    for path, recs in ((outfile, dcs_out), (single_path, single_out)):
        w = pysam.AlignmentFile(path, "wb", template=bam)
        for r in recs:
            w.write(r)
        w.close()
    stats = ("# === {} ===\nSSCS{} - Total reads: {}\nSSCS{} - Unmapped reads: {}\n"
             "SSCS{} - Secondary/Supplementary reads: {}\nDCS{} reads: {}\nSSCS{} singletons: {} \n").format(
        title, sc, totals[0], sc, totals[1], sc, 0, sc, len(dcs_out), sc, len(single_out))
    with open("%s.stats.txt" % prefix, "a") as f:
        f.write(stats)
    return dict(dcs=len(dcs_out), sscs_singletons=len(single_out))


def sc_stage(singleton, bedfile=None):
    base, rest = singleton.split(".singleton")[0], singleton.split(".singleton")[1]
    sbam = pysam.AlignmentFile(singleton, "rb")
    xbam = pysam.AlignmentFile("%s.sscs%s" % (base, rest), "rb")
    singles = FamilyBuilder()
    sscs = FamilyBuilder()
    resolved = collections.OrderedDict()
    by_sscs, by_single, uncorrected = [], [], []
    n_single_reads = 0
    n_processed = 0
    chrom_seen = "chrM"
    for key, chrom, start, end in regions_of(bedfile):
        if chrom is not None and chrom != chrom_seen:
            singles.size = collections.defaultdict(int)
            sscs = FamilyBuilder()
            chrom_seen = chrom
        reg = None if chrom is None else (start, end)
        n_single_reads += singles.feed(fetch(sbam, chrom, start, end), reg, duplex=True)[0]
        sscs.feed(fetch(xbam, chrom, start, end), reg, duplex=True)
        for mol in list(singles.entries):
            for k in singles.entries[mol]:
                n_processed += 1
                partner = complement_key(k)
                name = mol + ":1"
                own = singles.members[k][0]
                if partner in sscs.members:
                    seq, q = pair_vote(own, sscs.members[partner][0], gate=True)
                    by_sscs.append(new_record([own], seq, q, name))
                    del sscs.members[partner]
                    del singles.members[k]
                elif partner in singles.members:
                    seq, q = pair_vote(own, singles.members[partner][0], gate=True)
                    by_single.append(new_record([own], seq, q, name))
                    resolved[k] = partner
                    if partner in resolved:
                        del singles.members[k]
                        del singles.members[partner]
                        del resolved[k]
                        del resolved[partner]
                else:
                    uncorrected.append(own)
                    del singles.members[k]
            del singles.entries[mol]
    for suffix, recs in (("sscs.correction", by_sscs), ("singleton.correction", by_single),
                         ("uncorrected", uncorrected)):
        w = pysam.AlignmentFile("%s.%s.bam" % (base, suffix), "wb", template=sbam)
        for r in recs:
            w.write(r)
        w.close()
    if n_single_reads == 0:
        raise OracleError("ZeroDivisionError: empty singleton file")
    stats = ("# === Singleton Correction ===\nTotal singletons: {}\nSingleton Correction by SSCS: {}\n"
             "% Singleton Correction by SSCS: {}\nSingleton Correction by Singletons: {}\n"
             "% Singleton Correction by Singletons : {}\nUncorrected Singletons: {} \n").format(
        n_processed, len(by_sscs), len(by_sscs) / n_single_reads * 100, len(by_single),
        len(by_single) / n_single_reads * 100, len(uncorrected))
    with open("%s.stats.txt" % base, "a") as f:
        f.write(stats)
    return dict(sscs_correction=len(by_sscs), singleton_correction=len(by_single), uncorrected=len(uncorrected))


def consensus_pipeline(bam, c_output, bedfile="False", cutoff=0.7, bdelim="|", scorrect="True"):
    """ConsensusCruncher.py:127-346 with the oracle stages and the samtools stand-in."""
    ident = os.path.basename(bam).split(".bam", 1)[0]
    sd = os.path.join(c_output, ident)
    bed = None if bedfile == "False" else bedfile
    for sub in ("sscs", "dcs", "sscs_sc", "dcs_sc"):
        os.makedirs(os.path.join(sd, sub), exist_ok=True)
    p = lambda sub, name: os.path.join(sd, sub, "%s.%s" % (ident, name))  # noqa: E731
    sscs_stage(bam, p("sscs", "sscs.bam"), cutoff, bed, bdelim)
    out = dict(badreads=p("sscs", "badReads.bam"), read_families=p("sscs", "read_families.txt"))
    out["sscs"] = samtools_sort_index(p("sscs", "sscs.bam"))
    out["singleton"] = samtools_sort_index(p("sscs", "singleton.bam"))
    os.rename(p("sscs", "stats.txt"), p("dcs", "stats.txt"))
    dcs_stage(out["sscs"], p("dcs", "dcs.bam"), bed)
    out["dcs"] = samtools_sort_index(p("dcs", "dcs.bam"))
    out["sscs_singleton"] = samtools_sort_index(p("dcs", "sscs.singleton.bam"))
    stats = p("dcs", "stats.txt")
    if scorrect != "False":
        os.rename(stats, p("sscs", "stats.txt"))
        sc_stage(out["singleton"], bed)
        for name in ("sscs.correction", "singleton.correction", "uncorrected"):
            os.rename(p("sscs", name + ".bam"), p("sscs_sc", name + ".bam"))
            out[name.replace(".", "_")] = samtools_sort_index(p("sscs_sc", name + ".bam"))
        samtools_merge(p("sscs_sc", "sscs.sc.bam"), out["sscs"], out["sscs_correction"], out["singleton_correction"])
        out["sscs_sc"] = samtools_sort_index(p("sscs_sc", "sscs.sc.bam"))
        os.rename(p("sscs", "stats.txt"), p("dcs_sc", "stats.txt"))
        dcs_stage(out["sscs_sc"], p("dcs_sc", "dcs.sc.bam"), bed)
        out["dcs_sc"] = samtools_sort_index(p("dcs_sc", "dcs.sc.bam"))
        out["sscs_sc_singleton"] = samtools_sort_index(p("dcs_sc", "sscs.sc.singleton.bam"))
        samtools_merge(p("dcs_sc", "all.unique.dcs.bam"), out["dcs_sc"], out["sscs_sc_singleton"],
                       out["uncorrected"])
        out["all_unique"] = samtools_sort_index(p("dcs_sc", "all.unique.dcs.bam"))
        stats = p("dcs_sc", "stats.txt")
    out["stats"] = stats
    return out
