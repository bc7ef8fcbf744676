#!/usr/bin/env python3
"""Print the hottest functions of a cProfile dump written by ``scripts/mnist.py --cprofile PATH``.

Default output is the reference's view (/root/reference/mnist/read_stats.py: directories stripped, the
100 functions with the largest internal time).  Additive options: ``--sort`` (any pstats sort key, e.g.
``cumulative``, ``calls``) and the row count as a second positional argument.

  python3 scripts/read_stats.py mnist.prof            # top 100 by internal time
  python3 scripts/read_stats.py mnist.prof 30 --sort cumulative
"""
import argparse
import pstats


def show(path: str, rows: int = 100, sort: str = "time", stream=None) -> pstats.Stats:
    stats = pstats.Stats(path, stream=stream)
    stats.strip_dirs()
    stats.sort_stats(pstats.SortKey(sort) if sort in {k.value for k in pstats.SortKey} else sort)
    stats.print_stats(rows)
    return stats


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("path", help="cProfile output file")
    ap.add_argument("rows", nargs="?", type=int, default=100, help="functions to list (default 100)")
    ap.add_argument("--sort", default="time", help="pstats sort key (default: time = internal time)")
    a = ap.parse_args(argv)
    show(a.path, a.rows, a.sort)


if __name__ == "__main__":
    main()
