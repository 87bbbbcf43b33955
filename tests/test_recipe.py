"""Recipe parsing (CPU): the reference's recipe files (when /root/reference is mounted) and this
repo's configs parse into the expected modifiers / schemes; target matching semantics."""
import glob
import os

import pytest

from quantizers_amd.quantization import QuantizationArgs, preset_scheme
from quantizers_amd.recipe import AWQModifier, QuantizationModifier, is_match, parse_recipe

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/configs/recipes"


def test_repo_recipes_parse():
    for f in glob.glob(os.path.join(ROOT, "configs", "recipes", "*.yaml")):
        mods = parse_recipe(f)
        assert mods and all(isinstance(m, QuantizationModifier) for m in mods), f


def test_awq_g128():
    (m,) = parse_recipe(os.path.join(ROOT, "configs/recipes/awq_w4a16_g128.yaml"))
    assert isinstance(m, AWQModifier) and m.duo_scaling and m.n_grid == 20 and m.ignore == ["lm_head"]
    w = m.config_groups["group_0"].weights
    assert (w.num_bits, w.type, w.symmetric, w.group_size, w.strategy, w.observer) == (
        4, "int", True, 128, "group", "memoryless_minmax")


def test_mixed_recipe_two_modifiers():
    mods = parse_recipe(os.path.join(ROOT, "configs/recipes/mixed_fp8_block_awq_int4.yaml"))
    assert [type(m).__name__ for m in mods] == ["QuantizationModifier", "AWQModifier"]
    fp8 = mods[0].config_groups["group_0"]
    assert fp8.weights.strategy == "block" and fp8.weights.block_structure == [128, 128]
    assert len(mods[1].mappings) == 2


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference not mounted")
@pytest.mark.parametrize("name", ["recipe_awq_w4a16.yaml", "recipe_mixed_fp8_int4.yaml",
                                  "recipe_Minimax-M2.1-AWQ-MixedPrec.yaml", "recipe_Minimax-M2.1-Experts-only-AWQ.yaml",
                                  "recipe_MoE_RTN_NVFP4.yaml", "recipe_Dense_NVFP4.yaml"])
def test_reference_recipes(name):
    mods = parse_recipe(os.path.join(REF, name))
    assert mods
    if name == "recipe_awq_w4a16.yaml":  # M2 list shape
        (m,) = mods
        assert isinstance(m, AWQModifier) and m.config_groups["group_0"].weights.group_size == 32
    if name == "recipe_mixed_fp8_int4.yaml":  # M1 quirks normalised
        q, a = mods
        assert q.config_groups["group_0"].targets == ["re:.*self_attn\\.(k|q|o|v)_proj.*"]
        assert a.config_groups["group_0"].weights.num_bits == 4
    if name == "recipe_Minimax-M2.1-AWQ-MixedPrec.yaml":
        (m,) = mods
        assert m.config_groups["mlp_experts_projections"].weights.observer == "minmax"
        assert m.config_groups["self_attention_projections"].weights.type == "float"
        assert len(m.mappings) == 4


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference not mounted")
def test_autoround_is_out_of_scope():
    with pytest.raises(NotImplementedError):
        parse_recipe(os.path.join(REF, "recipe_AR_W4A16G32.yaml"))


def test_target_matching():
    assert is_match("model.layers.0.mlp.down_proj", "Linear", "Linear")
    assert is_match("model.layers.0.mlp.down_proj", "Linear", "re:.*mlp\\.(down_proj|gate_proj|up_proj)$")
    assert not is_match("model.layers.0.mlp.down_proj.x", "Linear", "re:.*down_proj$")
    assert is_match("lm_head", "Linear", "lm_head")
    assert is_match("model.layers.3.mlp.experts.7.gate_proj", "Linear", "re:.*mlp\\.experts\\.\\d+\\.(down_proj|gate_proj|up_proj)$")


def test_overlapping_groups_follow_target_precedence():
    """A module matched by several config groups takes the most specific target's group
    (compressed-tensors: exact name > regex > class name), not simply the first group."""
    from torch import nn
    from quantizers_amd.oneshot import resolve_schemes

    class Block(nn.Module):
        def __init__(self):
            super().__init__()
            self.q_proj = nn.Linear(8, 8, bias=False)
            self.down_proj = nn.Linear(8, 8, bias=False)
            self.up_proj = nn.Linear(8, 8, bias=False)

    model = nn.Module()
    model.layers = nn.ModuleList([Block()])
    recipe = {"s": {"m": {"QuantizationModifier": {"config_groups": {
        "group_0": {"targets": ["Linear"], "weights": {"num_bits": 8, "type": "int", "symmetric": True,
                                                       "strategy": "channel"}},
        "group_1": {"targets": ["re:.*down_proj$"], "weights": {"num_bits": 4, "type": "int", "symmetric": True,
                                                               "strategy": "group", "group_size": 8}},
        "group_2": {"targets": ["layers.0.up_proj", "re:.*up_proj$"],
                    "weights": {"num_bits": 4, "type": "int", "symmetric": False, "strategy": "group",
                                "group_size": 8}},
    }}}}}
    got = {k: (v[0].weights.num_bits, v[0].weights.symmetric) for k, v in resolve_schemes(model, parse_recipe(recipe)).items()}
    assert got == {"layers.0.q_proj": (8, True), "layers.0.down_proj": (4, True), "layers.0.up_proj": (4, False)}


def test_presets_and_validation():
    s = preset_scheme("W4A16", ["Linear"]).weights
    assert (s.num_bits, s.group_size, s.symmetric) == (4, 128, True)
    s = preset_scheme("NVFP4", ["Linear"]).weights
    assert s.is_nvfp4 and s.group_size == 16
    s = preset_scheme("MXFP4A16", ["Linear"]).weights
    assert s.is_mx and s.group_size == 32
    assert preset_scheme("FP8_BLOCK", ["Linear"]).weights.block_structure == [128, 128]
    with pytest.raises(ValueError):
        QuantizationArgs(num_bits=4, type="float", symmetric=False)
    with pytest.raises(ValueError):
        QuantizationArgs(num_bits=4, strategy="group")
    assert QuantizationArgs(num_bits=8, group_size=-1).strategy == "channel"
    with pytest.raises(ValueError):
        parse_recipe({"s": {"g": {"QuantizationModifier": {"scheme": "W4A16", "bogus": 1}}}})


def test_run_config(tmp_path):
    from quantizers_amd.config import load_run_config
    run = load_run_config(os.path.join(ROOT, "configs", "qwen3-4b-awq-g128.yaml"))
    assert run.resolve_recipe().endswith("configs/recipes/awq_w4a16_g128.yaml")
    assert run.output_dir() == "outputs/Qwen3-4B-awq_w4a16_g128"
    bad = tmp_path / "c.yaml"
    bad.write_text("model: {name: x}\nquantization: {recipe: nope.yaml}\n")
    with pytest.raises(ValueError):
        load_run_config(str(bad)).resolve_recipe()


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference not mounted")
def test_reference_run_configs_resolve():
    """Every run config the reference ships (configs/*.yaml) loads with the reference's path rules:
    recipe found and parsed, calibration-set file found and validated, output dir named as
    do_oneshot.py:114-121 names it; the AutoRound config raises NotImplementedError (out of scope)."""
    import glob
    from quantizers_amd.config import load_run_config
    files = sorted(glob.glob(os.path.join(os.path.dirname(REF), "*.yaml")))
    assert len(files) >= 6
    for f in files:
        run = load_run_config(f)
        assert run.calibration is not None, f
        recipe = run.resolve_recipe()
        if "-ar" in os.path.basename(f):
            with pytest.raises(NotImplementedError):
                parse_recipe(recipe)
            continue
        mods = parse_recipe(recipe)
        assert mods and all(m.config_groups or getattr(m, "mappings", None) is not None for m in mods), f
        assert run.output_dir().startswith("outputs/")
