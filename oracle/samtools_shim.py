"""samtools stand-in for the oracle and the fixture generator (TEST INFRASTRUCTURE).

sort_index (ConsensusCruncher.py:10-34): stable sort on samtools' coordinate key
tid<<32 | (pos+1)<<1 | is_reverse with tid read unsigned (unmapped last); ties
keep input order.  merge (ConsensusCruncher.py:262-266, 299-304): the same key,
ties in input-file order.  Pure Python over the pysam shim.
"""
import os
import struct
import sys

_SHIM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "shim")
if _SHIM not in sys.path:
    sys.path.insert(0, _SHIM)


def _sort_key(raw):
    tid, pos = struct.unpack_from("<ii", raw, 4)
    (flag,) = struct.unpack_from("<H", raw, 18)
    return (((tid & 0xffffffff) << 32) | ((pos + 1) & 0xffffffff) << 1 | ((flag >> 4) & 1))


def samtools_sort_index(bam):
    """sort_index() of ConsensusCruncher.py:10-34: X.bam -> X.sorted.bam (stable), X.bam removed."""
    from pysam import read_bam_file, write_bam_file
    header, raws = read_bam_file(bam)
    raws = sorted(raws, key=_sort_key)   # Python sort is stable
    out = bam.split(".bam", 1)[0] + ".sorted.bam"
    write_bam_file(out, header, raws)
    os.remove(bam)
    return out


def samtools_merge(out, *inputs):
    """samtools merge of coordinate-sorted inputs; ties keep input-file order."""
    from pysam import read_bam_file, write_bam_file
    header = None
    allr = []
    for fi, path in enumerate(inputs):
        h, raws = read_bam_file(path)
        header = header or h
        allr.extend((_sort_key(r), fi, k, r) for k, r in enumerate(raws))
    allr.sort(key=lambda x: (x[0], x[1], x[2]))
    write_bam_file(out, header, [x[3] for x in allr])
    return out


