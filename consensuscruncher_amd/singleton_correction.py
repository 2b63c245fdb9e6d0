#!/usr/bin/env python3
"""singleton_correction drop-in: same CLI and outputs as
ConsensusCruncher/singleton_correction.py (singleton_correction.py:118-139),
SSCS/singleton lookups and the corrected consensus on the GPU (libccamd)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--singleton", action="store", dest="singleton", help="input singleton BAM file",
                        required=True, type=str)
    parser.add_argument("--bedfile", action="store", dest="bedfile", required=False,
                        help="Bedfile containing coordinates to subdivide the BAM file")
    args = parser.parse_args(argv)
    from consensuscruncher_amd.stages import run_sc
    run_sc(args.singleton, bedfile=args.bedfile)


if __name__ == "__main__":
    start_time = time.time()
    main()
    print((time.time() - start_time) / 60)
