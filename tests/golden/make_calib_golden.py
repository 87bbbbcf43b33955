#!/usr/bin/env python3
"""Generate the calibration-data golden fixtures with the REFERENCE's own code (run in the build
container only, where /root/reference exists; the fixtures are committed, the reference is not):

* tests/golden/calib/cache_keys.json -- {yaml: {calibration_set section, key}}: CalibrationSet.compute_cache_key
  (src/quantizers/calibration_sets.py:409-462) of every reference calibration-set YAML plus
  tests/golden/calib/calib_set.yaml;
* tests/golden/calib/cache/<key> -- the reference-format parquet cache of calib_set.yaml, built
  by CalibrationSet.from_config + save_to_cache (calibration_sets.py:380-406, 689-707) from the
  reference's local test datasets (no network);
* tests/golden/calib/tokenizer/ -- a small byte-level BPE tokenizer with a chat template, trained
  deterministically on that cache's text (no pretrained tokenizer is available offline);
* tests/golden/calib/expected_ids.json -- CalibrationSet.get_tokenized(tokenizer) of the cache
  (calibration_sets.py:624-676: chat template, truncation to max_seq_length, no special tokens).
"""
import glob
import json
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "calib")
REF = "/root/reference"
CHAT_TEMPLATE = ("{% for m in messages %}<|{{ m['role'] }}|>\n{{ m['content'] }}\n{% endfor %}"
                 "{% if add_generation_prompt %}<|assistant|>\n{% endif %}")


def main():
    sys.path.insert(0, os.path.join(REF, "src"))
    from quantizers.calibration_sets import CalibrationSet, CalibrationSetConfig  # reference code (generator only)
    import yaml
    keys = {}
    vectors = {}  # input (the parsed calibration_set section) -> the reference's key
    for f in sorted(glob.glob(os.path.join(REF, "configs", "calibration_sets", "*.yaml"))):
        keys[os.path.basename(f)] = CalibrationSet.compute_cache_key(CalibrationSetConfig.from_file(f))
        vectors[os.path.basename(f)] = {"calibration_set": yaml.safe_load(open(f))["calibration_set"],
                                        "key": keys[os.path.basename(f)]}
    cfg_path = os.path.join(OUT, "calib_set.yaml")
    cfg = CalibrationSetConfig.from_file(cfg_path)
    keys["calib_set.yaml"] = CalibrationSet.compute_cache_key(cfg)
    vectors["calib_set.yaml"] = {"calibration_set": yaml.safe_load(open(cfg_path))["calibration_set"],
                                 "key": keys["calib_set.yaml"]}
    with open(os.path.join(OUT, "cache_keys.json"), "w") as f:
        json.dump(vectors, f, indent=1, sort_keys=True)
    cwd = os.getcwd()
    cache = os.path.join(OUT, "cache")
    shutil.rmtree(cache, ignore_errors=True)
    tmp = tempfile.mkdtemp()
    os.environ["HF_DATASETS_CACHE"] = os.path.join(tmp, "hf")
    os.chdir(REF)  # the dataset paths are relative to the reference checkout (read-only use)
    try:
        cs = CalibrationSet.from_config(cfg, cache_dir=cache)
        cs.save_to_cache()
    finally:
        os.chdir(cwd)
    # tokenizer trained on the cached text
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    from transformers import PreTrainedTokenizerFast
    texts = [m["content"] for row in cs._untokenized_calibration_set["formatted"] for m in row]
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tok.train_from_iterator(texts, trainers.BpeTrainer(vocab_size=600, special_tokens=["<pad>", "<eos>"],
                                                       initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    hf = PreTrainedTokenizerFast(tokenizer_object=tok, eos_token="<eos>", pad_token="<pad>")
    hf.chat_template = CHAT_TEMPLATE
    tdir = os.path.join(OUT, "tokenizer")
    shutil.rmtree(tdir, ignore_errors=True)
    hf.save_pretrained(tdir)
    from transformers import AutoTokenizer
    hf = AutoTokenizer.from_pretrained(tdir)
    ds = cs.get_tokenized(hf)
    ids = [list(map(int, r)) for r in ds["input_ids"]]
    with open(os.path.join(OUT, "expected_ids.json"), "w") as f:
        json.dump({"key": keys["calib_set.yaml"], "max_seq_length": cfg.max_seq_length, "input_ids": ids}, f)
    shutil.rmtree(tmp, ignore_errors=True)
    print(keys, len(ids), [len(i) for i in ids])


if __name__ == "__main__":
    main()
