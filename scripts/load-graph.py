#!/usr/bin/env python3
"""load-graph.py on the MI355X path: see khmer_amd/scripts.py (load_graph)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from khmer_amd.scripts import load_graph, run  # noqa: E402

if __name__ == "__main__":
    run(load_graph)
