"""Host-side mirror of the reference helpers (ConsensusCruncher/consensus_helper.py).

Only the parts the host needs live here: the bed-file region map (the shard map
for multi-GPU), and string-level versions of the key functions used to
document / test the packed-key semantics the GPU kernels implement
(cc_engine.hip: which_read, which_strand, duplex_key).  The per-read work itself
runs on the GPU; nothing here is on the data path.
"""
import collections


def bed_separator(bedfile):
    """consensus_helper.py:38-54: OrderedDict 'chr_arm' -> (start, end), file order;
    a repeated key keeps its first position and takes the last value."""
    coor = collections.OrderedDict()
    with open(bedfile) as f:
        for line in f:
            chr_arm = line.split('\t')
            chr_key = '{}_{}'.format(chr_arm[0], chr_arm[3])
            coor[chr_key] = (int(chr_arm[1]), int(chr_arm[2]))
    return coor


def region_list(bedfile):
    """[(key, contig, start, end)] in iteration order; contig = key.rsplit('_', 1)[0]
    (SSCS_maker.py:278-280)."""
    return [(k, k.rsplit('_', 1)[0], v[0], v[1]) for k, v in bed_separator(bedfile).items()]


def region_runs(regions, first_chr="chrM"):
    """Chromosome-run id per region: singleton_correction resets its SSCS dicts
    whenever the region's contig differs from the previous one, starting from
    last_chr = 'chrM' (singleton_correction.py:208-229)."""
    runs, run, last = [], 0, first_chr
    for _, chrom, _, _ in regions:
        if chrom != last:
            run += 1
            last = chrom
        runs.append(run)
    return runs


READ1 = (99, 83, 67, 115, 81, 97, 65, 113)
READ2 = (147, 163, 131, 179, 161, 145, 129, 177)


def which_read(flag):
    """consensus_helper.py:57-81 (without the prints)."""
    if flag in READ1:
        return 'R1'
    if flag in READ2:
        return 'R2'
    return None


def swap_barcode(barcode):
    """duplex_tag's barcode swap (consensus_helper.py:663-674)."""
    if '.' in barcode:
        i = barcode.index('.')
        return barcode[i + 1:] + '.' + barcode[:i]
    h = int(len(barcode) / 2)
    return barcode[h:] + barcode[:h]


def duplex_tag(tag):
    """consensus_helper.py:639-683."""
    s = tag.split('_')
    s[0] = swap_barcode(s[0])
    s[8] = 'R2' if s[8] == 'R1' else 'R1'
    return '_'.join(s)


def cutoff_pass(count, passed, cutoff):
    """SSCS_maker.py:153-155 in Python float semantics (the GPU evaluates the same
    IEEE double division)."""
    return passed != 0 and count / passed >= cutoff
