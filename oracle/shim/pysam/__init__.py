"""Test-only, pure-Python stand-in for the small part of pysam the reference uses.

TEST INFRASTRUCTURE — never imported by the product package.  pysam/htslib are
not installed in this image, so this module lets the reference's
own stage scripts (/root/reference/ConsensusCruncher/*.py) run in-process to
produce golden fixtures, and lets the tests decode BAMs written by the product
independently of the product's own native reader.

What it implements (SURVEY.md §8c "Full-stage oracle plan"):
  * BGZF read (gzip multi-member) / write (BC extra field, 0xff00-byte blocks,
    EOF marker), the BAM header and record codec;
  * ``AlignmentFile(path, "rb" | "wb", template=...)`` with ``fetch(until_eof=True)``
    and ``fetch(contig, start, stop)`` using htslib's overlap rule
    (``pos < stop and endpos > start``; endpos = pos + max(1, reference span),
    an unmapped read spans 1 — htslib ``bam_endpos``), ``write``, ``close``,
    ``mapped``, ``mate``, ``references``;
  * ``AlignedSegment`` with the attributes the reference touches
    (consensus_helper.py:308-619, SSCS_maker.py:81-168, DCS_maker.py:99-123,
    singleton_correction.py:61-111) and byte-level ``__eq__`` like pysam's
    ``compare()``.
Every ``fetch`` yields fresh objects, as pysam does.
"""
import struct
import zlib
import gzip
import array

__all__ = ["AlignmentFile", "AlignedSegment", "canonical_sam_line",
           "read_bam_file", "write_bam_file"]

CIGAR_OPS = "MIDNSHP=XB"
SEQ_NT16 = "=ACMGRSVTWYHKDBN"
_NT16_INDEX = {c: i for i, c in enumerate(SEQ_NT16)}
_BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


# --------------------------------------------------------------------------- BGZF
def bgzf_decompress(raw):
    return gzip.decompress(raw) if raw else b""


def bgzf_compress(data, level=6):
    out = bytearray()
    step = 0xff00
    for off in range(0, len(data), step):
        chunk = data[off:off + step]
        co = zlib.compressobj(level, zlib.DEFLATED, -15)
        cdata = co.compress(chunk) + co.flush()
        bsize = len(cdata) + 25
        out += struct.pack("<BBBBIBBHBBHH", 0x1f, 0x8b, 8, 4, 0, 0, 0xff, 6, 66, 67, 2, bsize)
        out += cdata
        out += struct.pack("<II", zlib.crc32(chunk) & 0xffffffff, len(chunk))
    out += _BGZF_EOF
    return bytes(out)


# --------------------------------------------------------------------------- header
class AlignmentHeader(object):
    def __init__(self, text, refs):
        self.text = text
        self.refs = list(refs)  # [(name, length)]

    def encode(self):
        t = self.text.encode()
        out = bytearray(b"BAM\x01")
        out += struct.pack("<i", len(t)) + t
        out += struct.pack("<i", len(self.refs))
        for name, ln in self.refs:
            nb = name.encode() + b"\x00"
            out += struct.pack("<i", len(nb)) + nb + struct.pack("<i", ln)
        return bytes(out)

    @property
    def references(self):
        return tuple(n for n, _ in self.refs)

    def get_tid(self, name):
        for i, (n, _) in enumerate(self.refs):
            if n == name:
                return i
        return -1


def _parse_header(buf):
    if buf[:4] != b"BAM\x01":
        raise ValueError("not a BAM file")
    (l_text,) = struct.unpack_from("<i", buf, 4)
    text = buf[8:8 + l_text].split(b"\x00", 1)[0].decode()
    off = 8 + l_text
    (n_ref,) = struct.unpack_from("<i", buf, off)
    off += 4
    refs = []
    for _ in range(n_ref):
        (l_name,) = struct.unpack_from("<i", buf, off)
        off += 4
        name = buf[off:off + l_name - 1].decode()
        off += l_name
        (l_ref,) = struct.unpack_from("<i", buf, off)
        off += 4
        refs.append((name, l_ref))
    return AlignmentHeader(text, refs), off


# --------------------------------------------------------------------------- aux
_AUX_INT = {"c": "<b", "C": "<B", "s": "<h", "S": "<H", "i": "<i", "I": "<I"}


def _parse_aux(data):
    tags = []
    off = 0
    n = len(data)
    while off + 3 <= n:
        tag = data[off:off + 2].decode()
        t = chr(data[off + 2])
        off += 3
        if t == "A":
            val = chr(data[off]); off += 1
        elif t in _AUX_INT:
            fmt = _AUX_INT[t]
            (val,) = struct.unpack_from(fmt, data, off); off += struct.calcsize(fmt)
        elif t == "f":
            (val,) = struct.unpack_from("<f", data, off); off += 4
        elif t in "ZH":
            end = data.index(b"\x00", off)
            val = data[off:end].decode(); off = end + 1
        elif t == "B":
            sub = chr(data[off]); (cnt,) = struct.unpack_from("<i", data, off + 1); off += 5
            fmt = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}[sub]
            sz = struct.calcsize(fmt)
            val = array.array(fmt, data[off:off + sz * cnt]); off += sz * cnt
            t = "B" + sub
        else:
            raise ValueError("bad aux type %r" % t)
        tags.append((tag, val, t))
    return tags


def _encode_aux(tags):
    out = bytearray()
    for tag, val, t in tags:
        out += tag.encode()
        if t == "A":
            out += b"A" + val.encode()
        elif t in _AUX_INT:
            out += t.encode() + struct.pack(_AUX_INT[t], val)
        elif t == "f":
            out += b"f" + struct.pack("<f", val)
        elif t in ("Z", "H"):
            out += t.encode() + str(val).encode() + b"\x00"
        elif t.startswith("B"):
            sub = t[1]
            out += b"B" + sub.encode() + struct.pack("<i", len(val)) + array.array(
                {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}[sub], val).tobytes()
        else:
            raise ValueError(t)
    return bytes(out)


def _int_type(v):
    if v >= 0:
        return "C" if v < 256 else ("S" if v < 65536 else "I")
    return "c" if v >= -128 else ("s" if v >= -32768 else "i")


def reg2bin(beg, end):
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


# --------------------------------------------------------------------------- record
class AlignedSegment(object):
    """The attribute subset of pysam.AlignedSegment used by the reference."""

    def __init__(self, header=None):
        self.query_name = None
        self.flag = 0
        self.reference_id = -1
        self.reference_start = -1
        self.mapping_quality = 0
        self.cigartuples = None
        self.next_reference_id = -1
        self.next_reference_start = -1
        self.template_length = 0
        self._seq = None
        self._qual = None
        self._tags = []
        self._bin = None
        self.header = header

    # ---- names / aliases
    @property
    def qname(self):
        return self.query_name

    @qname.setter
    def qname(self, v):
        self.query_name = v

    @property
    def cigar(self):
        return list(self.cigartuples) if self.cigartuples else []

    @cigar.setter
    def cigar(self, v):
        self.cigartuples = [tuple(x) for x in v] if v else None

    @property
    def cigarstring(self):
        if not self.cigartuples:
            return None
        return "".join("%d%s" % (ln, CIGAR_OPS[op]) for op, ln in self.cigartuples)

    @property
    def tlen(self):
        return self.template_length

    # ---- flags
    is_paired = property(lambda s: bool(s.flag & 0x1))
    is_proper_pair = property(lambda s: bool(s.flag & 0x2))
    is_unmapped = property(lambda s: bool(s.flag & 0x4))
    mate_is_unmapped = property(lambda s: bool(s.flag & 0x8))
    is_reverse = property(lambda s: bool(s.flag & 0x10))
    is_read1 = property(lambda s: bool(s.flag & 0x40))
    is_read2 = property(lambda s: bool(s.flag & 0x80))
    is_secondary = property(lambda s: bool(s.flag & 0x100))
    is_duplicate = property(lambda s: bool(s.flag & 0x400))
    is_supplementary = property(lambda s: bool(s.flag & 0x800))

    # ---- sequence / qualities (pysam: setting the sequence resets qualities)
    @property
    def query_sequence(self):
        return self._seq if self._seq else None

    @query_sequence.setter
    def query_sequence(self, s):
        self._seq = s if s else None
        self._qual = None

    @property
    def query_qualities(self):
        if not self._seq or self._qual is None:
            return None
        return self._qual

    @query_qualities.setter
    def query_qualities(self, q):
        self._qual = None if q is None else array.array("B", q)

    @property
    def query_length(self):
        return len(self._seq) if self._seq else 0

    def infer_query_length(self, always=False):
        if not self.cigartuples:
            return None
        ops = (0, 1, 4, 7, 8, 5) if always else (0, 1, 4, 7, 8)
        return sum(ln for op, ln in self.cigartuples if op in ops)

    @property
    def reference_end(self):
        if self.is_unmapped or not self.cigartuples:
            return None
        return self.reference_start + sum(ln for op, ln in self.cigartuples if op in (0, 2, 3, 7, 8))

    # ---- tags
    def get_tag(self, tag):
        for t, v, _ in self._tags:
            if t == tag:
                return v
        raise KeyError("tag '%s' not present" % tag)

    def has_tag(self, tag):
        return any(t == tag for t, _, _ in self._tags)

    def set_tag(self, tag, value, value_type=None):
        self._tags = [x for x in self._tags if x[0] != tag]
        if value is None:
            return
        if value_type is None:
            if isinstance(value, str):
                value_type = "Z"
            elif isinstance(value, float):
                value_type = "f"
            elif isinstance(value, int):
                value_type = _int_type(value)
            else:
                raise ValueError("unsupported tag value")
        self._tags.append((tag, value, value_type))

    def get_tags(self, with_value_type=False):
        return [(t, v, ty) if with_value_type else (t, v) for t, v, ty in self._tags]

    # ---- codec
    def _endpos(self):
        rl = 0
        if not (self.flag & 0x4) and self.cigartuples:
            rl = sum(ln for op, ln in self.cigartuples if op in (0, 2, 3, 7, 8))
        return self.reference_start + (rl if rl else 1)

    def encode(self):
        qn = (self.query_name or "*").encode() + b"\x00"
        cig = self.cigartuples or []
        seq = self._seq or ""
        l_seq = len(seq)
        sb = bytearray((l_seq + 1) // 2)
        for i, ch in enumerate(seq):
            code = _NT16_INDEX.get(ch.upper(), 15)
            if i & 1:
                sb[i >> 1] |= code
            else:
                sb[i >> 1] = code << 4
        if self._qual is None:
            qb = b"\xff" * l_seq
        else:
            qb = bytes(self._qual)
            if len(qb) != l_seq:
                raise ValueError("quality length != sequence length")
        bin_ = self._bin if self._bin is not None else reg2bin(
            max(self.reference_start, 0), max(self._endpos(), max(self.reference_start, 0) + 1))
        body = struct.pack("<iiBBHHHiiii", self.reference_id, self.reference_start, len(qn),
                           self.mapping_quality, bin_, len(cig), self.flag, l_seq,
                           self.next_reference_id, self.next_reference_start, self.template_length)
        body += qn
        body += b"".join(struct.pack("<I", (ln << 4) | op) for op, ln in cig)
        body += bytes(sb) + qb + _encode_aux(self._tags)
        return struct.pack("<i", len(body)) + body

    def _key(self):
        return (self.query_name, self.flag, self.reference_id, self.reference_start,
                self.mapping_quality, tuple(self.cigartuples or ()), self.next_reference_id,
                self.next_reference_start, self.template_length, self._seq,
                None if self._qual is None else bytes(self._qual), tuple((t, str(v), ty) for t, v, ty in self._tags))

    def compare(self, other):
        a, b = self._key(), other._key()
        return 0 if a == b else (-1 if repr(a) < repr(b) else 1)

    def __eq__(self, other):
        return isinstance(other, AlignedSegment) and self._key() == other._key()

    def __ne__(self, other):
        return not self.__eq__(other)

    def __hash__(self):
        return hash(self.query_name)

    def to_string(self):
        return canonical_sam_line(self)

    def __str__(self):
        return canonical_sam_line(self)


def _decode_record(buf, off, header):
    (block_size,) = struct.unpack_from("<i", buf, off)
    (tid, pos, l_qn, mapq, bin_, n_cig, flag, l_seq, mtid, mpos, tlen) = struct.unpack_from(
        "<iiBBHHHiiii", buf, off + 4)
    p = off + 36
    qn = buf[p:p + l_qn - 1].decode()
    p += l_qn
    cig = []
    for k in range(n_cig):
        (c,) = struct.unpack_from("<I", buf, p + 4 * k)
        cig.append((c & 0xf, c >> 4))
    p += 4 * n_cig
    nb = (l_seq + 1) // 2
    sraw = buf[p:p + nb]
    seq = "".join(SEQ_NT16[(sraw[i >> 1] >> (4 * (1 - (i & 1)))) & 0xf] for i in range(l_seq))
    p += nb
    qraw = buf[p:p + l_seq]
    p += l_seq
    end = off + 4 + block_size
    r = AlignedSegment(header)
    r.query_name = qn
    r.flag = flag
    r.reference_id = tid
    r.reference_start = pos
    r.mapping_quality = mapq
    r.cigartuples = cig if cig else None
    r.next_reference_id = mtid
    r.next_reference_start = mpos
    r.template_length = tlen
    r._seq = seq if l_seq else None
    r._qual = None if (l_seq == 0 or qraw[0] == 0xff) else array.array("B", qraw)
    r._tags = _parse_aux(buf[p:end])
    r._bin = bin_
    return r, end


def read_bam_file(path):
    """Return (header, [raw record byte strings]) for a BAM file."""
    with open(path, "rb") as f:
        buf = bgzf_decompress(f.read())
    header, off = _parse_header(buf)
    raws = []
    n = len(buf)
    while off < n:
        (bs,) = struct.unpack_from("<i", buf, off)
        raws.append(buf[off:off + 4 + bs])
        off += 4 + bs
    return header, raws


def write_bam_file(path, header, records, level=6):
    data = bytearray(header.encode())
    for r in records:
        data += r.encode() if isinstance(r, AlignedSegment) else r
    with open(path, "wb") as f:
        f.write(bgzf_compress(bytes(data), level))


class AlignmentFile(object):
    def __init__(self, path, mode="rb", template=None, header=None, **kw):
        self.filename = path
        self.mode = mode
        self._closed = False
        if mode.startswith("r"):
            self.header, self._raw = read_bam_file(path)
            self._records_cache = None
        else:
            if template is not None:
                self.header = template.header
            elif isinstance(header, AlignmentHeader):
                self.header = header
            else:
                raise ValueError("writer needs a template")
            self._out = []

    # ---- reading
    @property
    def references(self):
        return self.header.references

    def get_tid(self, name):
        return self.header.get_tid(name)

    def _decode(self, raw):
        r, _ = _decode_record(raw, 0, self.header)
        return r

    def fetch(self, contig=None, start=None, stop=None, until_eof=False, **kw):
        if contig is None:
            for raw in self._raw:
                yield self._decode(raw)
            return
        tid = self.header.get_tid(contig)
        if tid < 0:
            raise ValueError("invalid contig `%s`" % contig)
        start = 0 if start is None else start
        stop = (1 << 31) - 1 if stop is None else stop
        for raw in self._raw:
            (rtid, rpos) = struct.unpack_from("<ii", raw, 4)
            if rtid != tid or rpos >= stop:
                continue
            r = self._decode(raw)
            if r._endpos() > start:
                yield r

    def __iter__(self):
        return self.fetch(until_eof=True)

    @property
    def mapped(self):
        n = 0
        for raw in self._raw:
            (flag,) = struct.unpack_from("<H", raw, 18)
            n += 0 if flag & 0x4 else 1
        return n

    def mate(self, read):
        want = 0x80 if read.flag & 0x40 else 0x40
        for raw in self._raw:
            r = self._decode(raw)
            if r.query_name == read.query_name and (r.flag & want) and not (r.flag & 0x900):
                return r
        raise ValueError("mate not found")

    # ---- writing
    def write(self, read):
        self._out.append(read.encode())
        return 0

    def close(self):
        if self._closed:
            return
        self._closed = True
        if not self.mode.startswith("r"):
            write_bam_file(self.filename, self.header, self._out)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _fmt_aux(t, v, ty):
    if ty in _AUX_INT:
        return "%s:i:%d" % (t, v)
    if ty == "f":
        return "%s:f:%g" % (t, v)
    if ty.startswith("B"):
        return "%s:B:%s,%s" % (t, ty[1], ",".join(str(x) for x in v))
    return "%s:%s:%s" % (t, ty, v)


def canonical_sam_line(r):
    """One tab-separated SAM-like line (numeric tids, 0-based pos) with aux tags sorted.

    This is the unit of the parity comparison ("sorted record comparison",
    BASELINE.json north_star)."""
    qual = r.query_qualities
    qs = "*" if qual is None else "".join(chr(q + 33) for q in qual)
    tags = sorted(_fmt_aux(t, v, ty) for t, v, ty in r._tags)
    return "\t".join([str(r.query_name), str(r.flag), str(r.reference_id), str(r.reference_start),
                      str(r.mapping_quality), r.cigarstring or "*", str(r.next_reference_id),
                      str(r.next_reference_start), str(r.template_length), r.query_sequence or "*",
                      qs] + tags)


def sam_lines(path):
    """Canonical SAM lines of a BAM file, in file order."""
    header, raws = read_bam_file(path)
    return [canonical_sam_line(_decode_record(raw, 0, header)[0]) for raw in raws]
