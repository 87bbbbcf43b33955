"""``do_oneshot`` CLI: the reference's scripts/do_oneshot.py surface (same flags, same YAML keys,
same output-directory rule) on the MI355X path.

Reference flags (scripts/do_oneshot.py:47-79): --config, --output, --cache-dir, --log-file,
--debug.  Calibration data as in the reference (do_oneshot.py:137-169): the run config's
``calibration_set`` is looked up in ``--cache-dir`` under the reference's cache key and
tokenized with the model's tokenizer (``calibration.py``); the tokenizer is saved next to the
checkpoint (do_oneshot.py:198).  Offline additions (no Hub access in this environment):
--model-path (a local HF model directory instead of ``model.name``), --random-init (build
``model.name``'s architecture from a local config with random weights), --tokenizer (a local
tokenizer directory when the model has none), --calib-file (tokenized calibration set: .pt
tensor [N, S] or .jsonl rows with ``input_ids``) and --calib-random N,S (synthetic token ids).
Under torchrun rank 0 alone loads the model (the others hold a meta skeleton and receive each
decoder layer by broadcast, ``residency``), every rank runs the calibration (AWQ grid ratios /
expert searches split over the ranks), and each rank compresses and writes its own shards of the
checkpoint; rank 0 adds the index and config.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time
from typing import Optional

import torch

# under torchrun only rank 0 holds the model's host image (load_model); True: one copy per rank
RANK_COPIES = False


def setup_logging(log_file: Optional[str] = None, level: int = logging.INFO):
    handlers = [logging.StreamHandler(sys.stdout)]
    if log_file:
        handlers.append(logging.FileHandler(log_file))
    logging.basicConfig(level=level, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s",
                        handlers=handlers, force=True)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Calibration-based quantization entry point (MI355X)")
    p.add_argument("--config", type=str, required=True, help="Path to quantization configuration file")
    p.add_argument("--output", type=str, required=False, help="Output directory for quantized model")
    p.add_argument("--cache-dir", type=str, default="./cache", help="Directory to cache calibration sets")
    p.add_argument("--log-file", type=str, default=None, help="Path to log file (default: stdout only)")
    p.add_argument("--debug", action="store_true", help="Enable debug logging")
    p.add_argument("--model-path", type=str, default=None, help="local model directory (offline)")
    p.add_argument("--random-init", type=str, default=None,
                   help="HF config.json (file or dir) to build a random-weight model from")
    p.add_argument("--tokenizer", type=str, default=None, help="local tokenizer directory (offline)")
    p.add_argument("--calib-file", type=str, default=None)
    p.add_argument("--calib-random", type=str, default=None, help="N,S synthetic calibration tokens")
    p.add_argument("--max-seq-length", type=int, default=None)
    p.add_argument("--device", type=str, default=None)
    p.add_argument("--stateful-observers", action="store_true",
                   help="AWQ grid: minmax/static_minmax observers keep memory across grid points (DESIGN D7)")
    p.add_argument("--awq-dtype", choices=("bf16", "fp32"), default=None,
                   help="AWQ statistics / grid-scale dtype (DESIGN D8): bf16 = the activation dtype, as SURVEY "
                        "A.6 reads llmcompressor (default); fp32 = rounds 1-4")
    p.add_argument("--placement", choices=("auto", "resident", "layerwise"), default="auto",
                   help="AWQ: keep a host-loaded model on the GPU (resident), onload one decoder layer at a "
                        "time (layerwise, the reference's placement), or resident when it fits in half "
                        "the free HBM (auto)")
    return p.parse_args(argv)


def _calibration(args, run, vocab: int, tokenizer=None):
    """Tokenized calibration rows: --calib-file / --calib-random, else the run config's
    calibration set read from the reference-format cache in --cache-dir (do_oneshot.py:143-169)."""
    if args.calib_file:
        if args.calib_file.endswith(".pt"):
            t = torch.load(args.calib_file, weights_only=True)
            return [{"input_ids": r} for r in t]
        rows = []
        with open(args.calib_file) as f:
            for line in f:
                rows.append(json.loads(line))
        return rows
    if args.calib_random:
        n, s = (int(x) for x in args.calib_random.split(","))
        g = torch.Generator().manual_seed(42)  # reference shuffle seed (calibration_sets.py:618-619)
        return [{"input_ids": torch.randint(0, vocab, (s,), generator=g)} for _ in range(n)]
    if run.calibration:
        from . import calibration
        if tokenizer is None:
            raise ValueError("the calibration set needs the model's tokenizer: pass --model-path (a local model "
                             "directory with a tokenizer) or --tokenizer")
        t0 = time.time()
        rows = calibration.load_tokenized(run.calibration, args.cache_dir, tokenizer)
        logging.info("Loaded calibration set from cache %s (%d samples) in %.2f seconds",
                     calibration.cache_path(run.calibration, args.cache_dir), len(rows), time.time() - t0)
        return rows
    return None


def load_tokenizer(args, run):
    """The model's tokenizer (do_oneshot.py:94) from a local directory: --tokenizer, else
    --model-path, else ``model.name`` when it is a local directory; None when there is none."""
    from transformers import AutoTokenizer
    for path in (args.tokenizer, args.model_path, run.model.name):
        if path and os.path.isdir(path):
            try:
                return AutoTokenizer.from_pretrained(path)
            except (OSError, ValueError) as e:
                logging.debug("no tokenizer in %s: %s", path, e)
    return None


def load_model(args, run):
    """The model in bf16 on the host (do_oneshot.py:86-94).  Under torchrun only rank 0 loads the
    weights; the other ranks build a meta-device skeleton of the same architecture and receive
    each decoder layer by broadcast as the AWQ pass reaches it (``residency``): one host copy
    of the model for the whole job (RANK_COPIES = True restores one copy per rank)."""
    from transformers import AutoConfig, AutoModelForCausalLM
    if _rank() != 0 and not RANK_COPIES:
        cfg = AutoConfig.from_pretrained(args.random_init or args.model_path or run.model.name, trust_remote_code=True)
        with torch.device("meta"):
            return AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    if args.random_init:
        # offline stand-in for from_pretrained: random weights of the config's architecture, host
        # resident like a loaded checkpoint.  Initialised on the GPU (seconds; the CPU init of a
        # 4B model takes ~80 s) and copied to the host when it fits in half the free HBM.
        cfg = AutoConfig.from_pretrained(args.random_init)
        torch.manual_seed(0)
        with torch.device("meta"):
            n = sum(p.numel() for p in AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).parameters())
        dev = torch.device(args.device) if args.device else torch.device("cuda", torch.cuda.current_device())
        if n * 2 <= torch.cuda.mem_get_info(dev)[0] // 2:
            with torch.device(dev):
                model = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
            return model.to("cpu")
        return AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    path = args.model_path or run.model.name
    return AutoModelForCausalLM.from_pretrained(path, dtype=torch.bfloat16, low_cpu_mem_usage=True,
                                                trust_remote_code=True)


def _rank() -> int:
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _init_distributed(args) -> bool:
    """Under torchrun (WORLD_SIZE > 1): one process per GPU -- pin this rank's device and join the
    process group (RCCL) so oneshot splits the AWQ searches and save_compressed shards the
    compression over the ranks (rank 0 writes).  Returns True when this call created the group."""
    import torch
    import torch.distributed as dist
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1 or dist.is_initialized():
        return False
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("QZ_DIST_BACKEND", "nccl")  # gloo: rehearsal with ranks sharing a GPU
    if backend == "gloo":
        local %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if args.device is None:
        args.device = f"cuda:{local}"
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return True


def main(argv=None):
    args = parse_args(argv)
    setup_logging(args.log_file, logging.DEBUG if args.debug else logging.INFO)
    own_group = _init_distributed(args)
    from .config import load_run_config
    from .oneshot import oneshot
    from .compressor import save_compressed

    logging.info("Loading configuration from: %s", args.config)
    run = load_run_config(args.config)
    output_dir = args.output or run.output_dir()
    recipe_path = run.resolve_recipe()
    model = load_model(args, run)
    tokenizer = load_tokenizer(args, run)
    vocab = getattr(model.config, "vocab_size", 32000)
    dataset = _calibration(args, run, vocab, tokenizer)
    max_len = args.max_seq_length or (run.calibration or {}).get("max_seq_length", 2048)
    logging.info("Starting quantization")
    t0 = time.time()
    oneshot(model=model, recipe=recipe_path, dataset=dataset, max_seq_length=max_len,
            num_calibration_samples=len(dataset) if dataset else None, moe_calibrate_all_experts=True,
            device=args.device, stateful_observers=args.stateful_observers,
            device_resident={"auto": None, "resident": True, "layerwise": False}[args.placement],
            awq_dtype=args.awq_dtype)
    logging.info("Completed quantization in %.2f seconds", time.time() - t0)
    if _rank() == 0:
        os.makedirs("outputs", exist_ok=True)
    logging.info("Saving quantized model to: %s", output_dir)
    t0 = time.time()
    save_compressed(model, output_dir)  # under torchrun each rank writes its own shards
    if tokenizer is not None and _rank() == 0:
        tokenizer.save_pretrained(output_dir)
    logging.info("Saved quantized model in %.2f seconds", time.time() - t0)
    logging.info("SUCCESS: Quantized model saved in %s", output_dir)
    if own_group:
        import torch.distributed as dist
        dist.destroy_process_group()
    return output_dir


if __name__ == "__main__":
    main()
