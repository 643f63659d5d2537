"""bench.py --engine-factory hooks (test infrastructure: the CPU oracle stands in for the GPU engine
so that the multi-rank host path of bench.py runs in a CPU-only container)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))


def oracle_lib():
    import oracle
    return oracle.lib()
