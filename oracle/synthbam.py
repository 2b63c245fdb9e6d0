"""Write a consensuscruncher_amd.synth Batch as BAM through the pysam shim.

TEST INFRASTRUCTURE: used to build golden-fixture inputs independently of the
product's native BAM writer.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if os.path.join(HERE, "shim") not in sys.path:
    sys.path.insert(0, os.path.join(HERE, "shim"))

import pysam  # noqa: E402  (shim)
from consensuscruncher_amd import synth  # noqa: E402

_OPS = {c: i for i, c in enumerate("MIDNSHP=XB")}


def _parse_cigar(s):
    out, num = [], ""
    for ch in s:
        if ch.isdigit():
            num += ch
        else:
            out.append((_OPS[ch], int(num)))
            num = ""
    return out


def batch_records(batch, delim="|"):
    header = pysam.AlignmentHeader(synth.sam_header_text(batch), list(zip(batch.names, batch.lens)))
    cig = [_parse_cigar(s) for s in batch.cigar_table]
    recs = []
    for i in range(batch.n):
        r = pysam.AlignedSegment(header)
        r.query_name = synth.qname_of(batch, i, delim)
        r.flag = int(batch.flag[i])
        r.reference_id = int(batch.tid[i])
        r.reference_start = int(batch.pos[i])
        r.mapping_quality = int(batch.mapq[i])
        c = int(batch.cig[i])
        r.cigartuples = cig[c] if c >= 0 else None
        r.next_reference_id = int(batch.mtid[i])
        r.next_reference_start = int(batch.mpos[i])
        r.template_length = int(batch.tlen[i])
        r.query_sequence = batch.seq[i].tobytes().decode()
        r.query_qualities = batch.qual[i]
        r.set_tag("RG", batch.rg_table[int(batch.rg[i])])
        recs.append(r)
    return header, recs


def write_batch(batch, path, level=6, delim="|"):
    header, recs = batch_records(batch, delim)
    pysam.write_bam_file(path, header, recs, level)
    return path
