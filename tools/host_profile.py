#!/usr/bin/env python3
"""cProfile of the drop-in path on a tiny scene (host overhead hunting)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import host_overhead as H  # noqa: E402

if __name__ == "__main__":
    pr = cProfile.Profile()
    pr.enable()
    H.main()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
