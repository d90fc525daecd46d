"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the RT-DETRv2 /detect hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import anything under oracle/. The product path (spotter_amd/) never does: it
runs on the HIP extension or fails loudly.
"""
