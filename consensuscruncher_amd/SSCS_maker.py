#!/usr/bin/env python3
"""SSCS_maker drop-in: same CLI and outputs as ConsensusCruncher/SSCS_maker.py
(SSCS_maker.py:183-226), consensus computed on the GPU (libccamd)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class SmartFormatter(argparse.HelpFormatter):
    def _split_lines(self, text, width):
        if text.startswith('R|'):
            return text[2:].splitlines()
        return argparse.HelpFormatter._split_lines(self, text, width)


def main(argv=None):
    parser = argparse.ArgumentParser(formatter_class=SmartFormatter)
    parser.add_argument("--cutoff", action="store", dest="cutoff", type=float, required=True,
                        help="R|Proportion of nucleotides at a given position in a\nsequence required to be identical"
                             " to form a consensus\n(Recommendation: 0.7 - based on previous literature\nKennedy et al.)\n"
                             "   Example (--cutoff = 0.7):\n"
                             "       Four reads (readlength = 10) are as follows:\n"
                             "       Read 1: ACTGATACTT\n"
                             "       Read 2: ACTGAAACCT\n"
                             "       Read 3: ACTGATACCT\n"
                             "       Read 4: ACTGATACTT\n"
                             "   The resulting SSCS is: ACTGATACNT")
    parser.add_argument("--infile", action="store", dest="infile", help="Input BAM file", required=True)
    parser.add_argument("--outfile", action="store", dest="outfile", help="Output SSCS BAM file", required=True)
    parser.add_argument("--bdelim", action="store", dest="bdelim", default="|",
                        help="Delimiter to differentiate barcodes from read name, default: '|'")
    parser.add_argument("--bedfile", action="store", dest="bedfile", required=False,
                        help="Bedfile containing coordinates to subdivide the BAM file (Recommendation: cytoband.txt - "
                             "See bed_separator.R for making your own bed file based on a target panel/specific "
                             "coordinates)")
    args = parser.parse_args(argv)
    from consensuscruncher_amd.stages import run_sscs
    run_sscs(args.infile, args.outfile, args.cutoff, bedfile=args.bedfile, bdelim=args.bdelim)


if __name__ == "__main__":
    start_time = time.time()
    main()
    print((time.time() - start_time) / 60)
