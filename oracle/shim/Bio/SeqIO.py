"""SeqIO.parse(handle, "fastq") / SeqIO.write(record, handle, "fastq") (TEST INFRASTRUCTURE).

Follows Biopython's documented FASTQ (Sanger) behaviour for the 4-line records the reference's
test data holds: the title is the header line after '@' without trailing whitespace, id = the
title up to the first whitespace, description = the title; qualities are phred = ord(c) - 33.
On writing, the title line is the description when its first word is the id, else
"id description"; the '+' line is bare.
"""


class Seq(str):
    def __getitem__(self, k):
        return Seq(str.__getitem__(self, k))


class SeqRecord(object):
    def __init__(self, seq, id, description, qual):
        self.seq = Seq(seq)
        self.id = id
        self.name = id
        self.description = description
        self.letter_annotations = {"phred_quality": list(qual)}

    def __getitem__(self, k):
        if not isinstance(k, slice):
            raise TypeError("only slices are supported by the stand-in")
        return SeqRecord(str(self.seq)[k], self.id, self.description, self.letter_annotations["phred_quality"][k])


def parse(handle, fmt):
    if fmt != "fastq":
        raise ValueError("the stand-in reads FASTQ only")
    while True:
        title = handle.readline()
        if not title:
            return
        title = title.rstrip()
        if not title:
            continue
        if not title.startswith("@"):
            raise ValueError("Records in Fastq files should start with '@' character")
        title = title[1:]
        seq = handle.readline().rstrip()
        plus = handle.readline()
        if not plus.startswith("+"):
            raise ValueError("the stand-in expects 4-line FASTQ records")
        qual = handle.readline().rstrip("\r\n")
        if len(qual) != len(seq):
            raise ValueError("Lengths of sequence and quality values differs")
        words = title.split(None, 1)
        yield SeqRecord(seq, words[0] if words else "", title, [ord(c) - 33 for c in qual])


def write(records, handle, fmt):
    if fmt != "fastq":
        raise ValueError("the stand-in writes FASTQ only")
    if isinstance(records, SeqRecord):
        records = [records]
    n = 0
    for r in records:
        d = r.description
        if d and d.split(None, 1)[0] == r.id:
            title = d
        elif d:
            title = "%s %s" % (r.id, d)
        else:
            title = r.id
        q = "".join(chr(x + 33) for x in r.letter_annotations["phred_quality"])
        handle.write("@%s\n%s\n+\n%s\n" % (title, str(r.seq), q))
        n += 1
    return n
