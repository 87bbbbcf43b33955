#!/usr/bin/env python3
"""AWQ oneshot on an N-layer Qwen3-4B-shaped model (bench.py's awq_oneshot_layers), for
rocprofv3 breakdowns: python scripts/awq_e2e.py [layers] [n_seq] [seq]."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ns = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    sq = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
    print(json.dumps(bench.awq_oneshot_layers(torch.device("cuda:0"), n, ns, sq)), flush=True)
