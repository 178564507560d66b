"""Benchmark legs behind bench.py (C4 batch, C5 skew) and the CPU-baseline helper.

Not part of the product package: the cpu_baseline legs load the oracle (oracle/cpu_ref), which
only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use.
"""
