#!/usr/bin/env python3
"""Calibration-based quantization entry point (MI355X-native drop-in for the reference's
scripts/do_oneshot.py; same flags).  Usage:
    python scripts/do_oneshot.py --config configs/test-quantize_qwen3-4b-awq.yaml [--random-init DIR]
"""
import os
import sys

os.environ.setdefault("TOKENIZERS_PARALLELISM", "false")
os.environ.setdefault("PYTORCH_ALLOC_CONF", "expandable_segments:True,max_split_size_mb:512")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from quantizers_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    main()
