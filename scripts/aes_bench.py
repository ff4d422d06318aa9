"""AES-128 (fixed key) throughput probe of the device T-table implementation."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dash_amd.native import native  # noqa: E402

n = native()
for blocks in (512, 1024, 2048):
    ms, rate = n.hip_aes_bench(blocks, 2000)
    print(f"aes_bench blocks={blocks} ms={ms:.2f} rate={rate / 1e9:.1f} G AES/s", flush=True)
