"""The CLI's calibration data path against fixtures made by the reference's OWN code
(tests/golden/make_calib_golden.py, run in the build container): the cache key of every
reference calibration-set config, and the tokenized rows of a reference-written parquet cache."""
import json
import os
import shutil

import pytest
import yaml

from quantizers_amd import calibration, cli
from quantizers_amd.config import load_run_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "calib")


def test_cache_keys_match_reference():
    vectors = json.load(open(os.path.join(GOLD, "cache_keys.json")))
    assert len(vectors) >= 8
    for name, v in vectors.items():
        assert calibration.compute_cache_key({"calibration_set": v["calibration_set"]}) == v["key"], name


def test_cache_key_ignores_order_and_formatter_params():
    v = json.load(open(os.path.join(GOLD, "cache_keys.json")))["calib_set.yaml"]
    c = dict(v["calibration_set"])
    c["datasets"] = list(reversed(c["datasets"]))
    c["datasets"][0] = dict(c["datasets"][0], formatter_params={"prefix": "x"})
    assert calibration.compute_cache_key(c) == v["key"]
    c["seed"] = 7
    assert calibration.compute_cache_key(c) != v["key"]
    c = dict(v["calibration_set"], datasets=[dict(v["calibration_set"]["datasets"][0], num_samples="all")])
    assert calibration.compute_cache_key(c).endswith("-length_TBD.parquet")


@pytest.mark.parametrize("bad,msg", [({"split": None}, "Split is required"), ({"columns": []}, "columns list"),
                                     ({"num_samples": 0}, "num_samples must be"), ({"formatter": ""}, "formatter")])
def test_validation_errors_like_reference(bad, msg):
    d = {"dataset": "x", "split": "train", "columns": ["a"], "formatter": "raw_text", "num_samples": 1}
    d.update(bad)
    with pytest.raises(ValueError, match=msg):
        calibration.normalise({"calibration_set": {"datasets": [d]}})


def _run_config(tmp_path):
    shutil.copy(os.path.join(GOLD, "calib_set.yaml"), tmp_path / "calib_set.yaml")
    (tmp_path / "recipes").mkdir()
    shutil.copy(os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g32.yaml"), tmp_path / "recipes" / "r.yaml")
    cfg = {"model": {"name": "Qwen/Qwen3-4B"}, "quantization": {"recipe": "r.yaml"},
           "calibration_set": "calib_set.yaml"}
    (tmp_path / "run.yaml").write_text(yaml.safe_dump(cfg))
    return str(tmp_path / "run.yaml")


def test_cli_reads_reference_cache(tmp_path):
    """do_oneshot's data path: run config -> calibration set -> cache key in --cache-dir ->
    parquet rows -> chat template + truncation -> the reference's token ids."""
    cfgp = _run_config(tmp_path)
    args = cli.parse_args(["--config", cfgp, "--cache-dir", os.path.join(GOLD, "cache"),
                           "--tokenizer", os.path.join(GOLD, "tokenizer")])
    run = load_run_config(cfgp)
    assert run.calibration["max_seq_length"] == 48
    tok = cli.load_tokenizer(args, run)
    rows = cli._calibration(args, run, 600, tok)
    want = json.load(open(os.path.join(GOLD, "expected_ids.json")))
    assert [r["input_ids"] for r in rows] == want["input_ids"]
    assert all(len(r["input_ids"]) <= 48 for r in rows)


def test_cli_cache_miss_and_missing_tokenizer(tmp_path):
    cfgp = _run_config(tmp_path)
    run = load_run_config(cfgp)
    args = cli.parse_args(["--config", cfgp, "--cache-dir", str(tmp_path / "empty"),
                           "--tokenizer", os.path.join(GOLD, "tokenizer")])
    with pytest.raises(FileNotFoundError, match="Cache not found"):
        cli._calibration(args, run, 600, cli.load_tokenizer(args, run))
    args = cli.parse_args(["--config", cfgp, "--cache-dir", os.path.join(GOLD, "cache")])
    with pytest.raises(ValueError, match="tokenizer"):
        cli._calibration(args, run, 600, cli.load_tokenizer(args, run))


def test_tokenizer_saved_next_to_checkpoint(tmp_path):
    """do_oneshot.py:198: the tokenizer goes beside the checkpoint (a model directory given with
    --model-path carries its tokenizer)."""
    mdir = tmp_path / "model"
    shutil.copytree(os.path.join(GOLD, "tokenizer"), mdir)
    cfgp = _run_config(tmp_path)
    args = cli.parse_args(["--config", cfgp, "--model-path", str(mdir)])
    tok = cli.load_tokenizer(args, load_run_config(cfgp))
    assert tok is not None
    out = tmp_path / "out"
    tok.save_pretrained(str(out))
    assert (out / "tokenizer.json").exists() and (out / "tokenizer_config.json").exists()
