#!/usr/bin/env python3
"""DCS_maker drop-in: same CLI and outputs as ConsensusCruncher/DCS_maker.py
(DCS_maker.py:130-152), duplex pairing and consensus on the GPU (libccamd)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--infile", action="store", dest="infile", help="Input BAM file", required=True)
    parser.add_argument("--outfile", action="store", dest="outfile", help="Output BAM file", required=True)
    parser.add_argument("--bedfile", action="store", dest="bedfile", required=False,
                        help="Bedfile containing coordinates to subdivide the BAM file")
    args = parser.parse_args(argv)
    from consensuscruncher_amd.stages import run_dcs
    run_dcs(str(args.infile), str(args.outfile), bedfile=args.bedfile)


if __name__ == "__main__":
    main()
