#!/usr/bin/env python3
"""Pretty-print a pstats file written by ``scripts/mnist.py --cprofile PATH`` (reference:
/root/reference/mnist/read_stats.py: top 100 by internal time)."""
import pstats
import sys
from pstats import SortKey

if __name__ == "__main__":
    p = pstats.Stats(sys.argv[1])
    p.strip_dirs().sort_stats(SortKey.TIME).print_stats(int(sys.argv[2]) if len(sys.argv) > 2 else 100)
