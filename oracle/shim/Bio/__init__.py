"""Test-only, pure-Python stand-in for the part of Biopython the reference's
extract_barcodes.py uses (SeqIO FASTQ parse/write, SeqRecord slicing).

TEST INFRASTRUCTURE — never imported by the product.  Biopython is not installed
in this image, so this lets the reference's own extract_barcodes.py run unmodified
in this container (oracle/refrun.py) to produce golden fixtures for the product's
native UMI extraction (consensuscruncher_amd/extract_barcodes.py).
"""
