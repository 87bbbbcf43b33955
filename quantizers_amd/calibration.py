"""Calibration-set cache reader: the CLI consumes the parquet cache the reference's tooling writes.

The reference builds its calibration set from Hugging Face Hub datasets (network), formats every
row into chat messages and caches the untokenized result as ``<cache_dir>/<key>.parquet``
(src/quantizers/calibration_sets.py: ``compute_cache_key`` :409-462, ``save_to_cache`` :689-707,
``is_cached`` / ``from_cache`` :312-377), then tokenizes it with the model's chat template
(``_tokenize_row`` / ``get_tokenized`` :624-676) and hands the token ids to ``oneshot``
(scripts/do_oneshot.py:143-169).  Building the set needs the Hub (out of scope offline); this
module restates the cache key, reads a cache the reference produced, and tokenizes it the same
way, so ``scripts/do_oneshot.py --cache-dir`` finds and uses the same file.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Any, Dict, List, Optional, Union

DEFAULTS = {"max_seq_length": 4096, "shuffle": True, "seed": 42}


def normalise(data: Dict[str, Any]) -> Dict[str, Any]:
    """``calibration_set:`` YAML section (or the whole file) -> dict with the reference's defaults
    (CalibrationSetConfig.from_dict, calibration_sets.py:208-224) and its validation errors
    (DatasetEntryConfig.from_dict, :70-107)."""
    if "calibration_set" in data:
        data = data["calibration_set"]
    out = {k: data.get(k, v) for k, v in DEFAULTS.items()}
    dss = []
    for d in data.get("datasets", []) or []:
        if not d.get("dataset"):
            raise ValueError("Dataset is required in calibration entry")
        if not d.get("split"):
            raise ValueError("Split is required in calibration entry")
        cols = d.get("columns", [])
        if not isinstance(cols, list):
            raise ValueError(f"columns must be a list, got {type(cols)}")
        if not cols:
            raise ValueError("columns list cannot be empty")
        if not d.get("formatter"):
            raise ValueError("formatter is required in calibration entry")
        n = d.get("num_samples")
        if n is None:
            raise ValueError("num_samples is required in calibration entry")
        if not (n == "all" or (isinstance(n, int) and not isinstance(n, bool) and n > 0)):
            raise ValueError("num_samples must be a positive integer or 'all'")
        dss.append({"dataset": d["dataset"], "split": d["split"], "subset": d.get("subset"), "columns": list(cols),
                    "formatter": d["formatter"], "num_samples": n, "streaming": d.get("streaming", False),
                    "formatter_params": d.get("formatter_params") or {}})
    if not dss:
        raise ValueError("Calibration set must have at least one dataset")
    out["datasets"] = dss
    return out


def compute_cache_key(calib: Dict[str, Any]) -> str:
    """``<first 7 hex of sha256(canonical json)>-<total samples>.parquet``: the canonical form is
    the sorted per-dataset tuples (dataset, split, subset, num_samples, columns, formatter) plus
    max_seq_length / shuffle / seed (calibration_sets.py:409-462; formatter_params are not part of
    the key, as in the reference)."""
    calib = normalise(calib)
    rows = [[d["dataset"], d["split"], d["subset"], d["num_samples"], list(d["columns"]), d["formatter"]]
            for d in calib["datasets"]]
    rows.sort(key=lambda x: (x[0], x[1], str(x[2])))
    canonical = {"datasets": rows, "max_seq_length": calib["max_seq_length"], "shuffle": calib["shuffle"],
                 "seed": calib["seed"]}
    prefix = hashlib.sha256(json.dumps(canonical, sort_keys=True).encode()).hexdigest()[:7]
    total, tbd = 0, False
    for d in calib["datasets"]:
        if d["num_samples"] == "all":
            tbd = True
            break
        total += d["num_samples"]
    return f"{prefix}-{'length_TBD' if tbd else total}.parquet"


def cache_path(calib: Dict[str, Any], cache_dir: str) -> str:
    return os.path.join(cache_dir, compute_cache_key(calib))


def is_cached(calib: Dict[str, Any], cache_dir: str) -> bool:
    return os.path.exists(cache_path(calib, cache_dir))


def load_cached(calib: Dict[str, Any], cache_dir: str) -> List[List[Dict[str, str]]]:
    """The cached rows' chat messages (column ``formatted``), in file order."""
    import pyarrow.parquet as pq
    path = cache_path(calib, cache_dir)
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"Cache not found for configuration. Expected cache file: {path}.  Building a calibration "
            f"set needs the Hugging Face Hub (out of scope offline): build the cache with the reference's "
            f"tooling, or pass --calib-file / --calib-random")
    rows = pq.read_table(path).to_pylist()
    if not rows:
        raise ValueError(f"Cache found but empty: {path}")
    return [r["formatted"] for r in rows]


def tokenize(messages: List[List[Dict[str, str]]], tokenizer, max_seq_length: int) -> List[Dict[str, Any]]:
    """Chat template -> token ids, truncated to ``max_seq_length``, no special tokens added
    (calibration_sets.py:624-647)."""
    out = []
    for m in messages:
        text = tokenizer.apply_chat_template(m, tokenize=False)
        t = tokenizer(text, padding=False, max_length=max_seq_length, truncation=True, add_special_tokens=False)
        out.append({"input_ids": list(t["input_ids"]), "attention_mask": list(t["attention_mask"])})
    return out


def load_tokenized(calib: Union[Dict[str, Any], None], cache_dir: str, tokenizer,
                   max_seq_length: Optional[int] = None) -> List[Dict[str, Any]]:
    """The CLI's calibration data: the reference-format cache for ``calib``, tokenized."""
    calib = normalise(calib)
    return tokenize(load_cached(calib, cache_dir), tokenizer, max_seq_length or calib["max_seq_length"])
