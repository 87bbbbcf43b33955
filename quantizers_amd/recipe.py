"""Recipe parsing: the reference's YAML recipes (configs/recipes/*.yaml) -> modifier objects.

Accepts every shape the reference's recipes use (SURVEY.md §2 notes M1/M2):

* ``<stage>: <group>: {ModifierName: {args}}``  (recipe_Dense_NVFP4.yaml:7-12,
  recipe_Minimax-M2.1-AWQ-MixedPrec.yaml:20-59, recipe_mixed_fp8_int4.yaml:7-36)
* top-level ``quantization_scheme`` + ``modifiers: [{name: X, ...}]``
  (recipe_awq_w4a16.yaml:7-31, quirk M2)
* M1 quirks of recipe_mixed_fp8_int4.yaml: a target written as the unquoted YAML scalar
  ``r"re:..."`` (the ``r"`` prefix and closing quote become part of the string) and config
  groups nested under an extra key instead of ``config_groups`` -- normalised with a warning,
  following the well-formed equivalent in scripts/quantization_multiple_modifiers.py:58-91.

Registry names are accepted verbatim: modifiers ``AWQModifier``, ``QuantizationModifier``
(``GPTQModifier``/``AutoRoundModifier`` are recognised and rejected as out of scope);
observers ``memoryless_minmax``, ``minmax``, ``static_minmax``; preset schemes (W4A16,
W4A16_ASYM, W8A16, W8A8, FP8, FP8_DYNAMIC, FP8_BLOCK, NVFP4, NVFP4A16, MXFP4, MXFP4A16).
"""
from __future__ import annotations

import logging
import os
import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union

import yaml

from .quantization import QuantizationArgs, QuantizationScheme, preset_scheme

log = logging.getLogger(__name__)

OBSERVERS = ("memoryless_minmax", "minmax", "static_minmax", "memoryless")
_ARG_KEYS = {"num_bits", "type", "symmetric", "group_size", "strategy", "block_structure", "dynamic", "actorder",
             "observer", "observer_kwargs", "scale_dtype", "zp_dtype"}


def _clean_target(t: str) -> str:
    """M1: unquoted YAML ``r"re:..."`` keeps the python raw-string wrapper; strip it."""
    s = str(t).strip()
    m = re.fullmatch(r'r(["\'])(.*)\1', s)
    if m:
        log.warning("recipe target %r looks like a python raw string; using %r", s, m.group(2))
        s = m.group(2)
    return s


def _targets(v) -> List[str]:
    if v is None:
        return []
    if isinstance(v, str):
        return [_clean_target(v)]
    return [_clean_target(x) for x in v]


def _args(d: Optional[Dict[str, Any]]) -> Optional[QuantizationArgs]:
    if d is None:
        return None
    unknown = set(d) - _ARG_KEYS
    if unknown:
        raise ValueError(f"unknown QuantizationArgs fields {sorted(unknown)}")
    a = QuantizationArgs(**{k: v for k, v in d.items()})
    if a.observer is not None and a.observer not in OBSERVERS:
        raise ValueError(f"observer {a.observer!r} not supported (have {OBSERVERS})")
    return a


def _scheme_from_group(name: str, g: Dict[str, Any]) -> QuantizationScheme:
    if "targets" not in g:
        raise ValueError(f"config group {name} has no targets")
    return QuantizationScheme(targets=_targets(g["targets"]), weights=_args(g.get("weights")),
                              input_activations=_args(g.get("input_activations")),
                              output_activations=_args(g.get("output_activations")), format=g.get("format"))


def _looks_like_groups(v: Any) -> bool:
    return isinstance(v, dict) and v and all(isinstance(x, dict) and "targets" in x for x in v.values())


@dataclass
class QuantizationModifier:
    """llmcompressor ``QuantizationModifier`` (RTN: observe -> qparams -> quantize)."""

    config_groups: Dict[str, QuantizationScheme] = field(default_factory=dict)
    ignore: List[str] = field(default_factory=list)

    name = "QuantizationModifier"


@dataclass
class AWQMapping:
    smooth_layer: str
    balance_layers: List[str]


@dataclass
class AWQModifier(QuantizationModifier):
    """llmcompressor ``AWQModifier``: activation-aware scale search, then quantization."""

    mappings: Optional[List[AWQMapping]] = None
    duo_scaling: bool = True
    n_grid: int = 20

    name = "AWQModifier"


def _schemes(args: Dict[str, Any], default_scheme: Optional[QuantizationScheme]) -> Dict[str, QuantizationScheme]:
    groups: Dict[str, QuantizationScheme] = {}
    cg = args.pop("config_groups", None)
    if cg:
        for k, g in cg.items():
            groups[k] = _scheme_from_group(k, g)
    scheme = args.pop("scheme", None)
    targets = _targets(args.pop("targets", None))
    if scheme is not None:
        if isinstance(scheme, str):
            groups[f"group_{len(groups)}"] = preset_scheme(scheme, targets or ["Linear"])
        elif isinstance(scheme, dict):
            for preset, tg in scheme.items():
                groups[f"group_{len(groups)}"] = preset_scheme(preset, _targets(tg))
        else:
            raise ValueError(f"bad scheme {scheme!r}")
    elif targets and not groups and default_scheme is not None:
        groups["group_0"] = QuantizationScheme(targets=targets, weights=default_scheme.weights,
                                               input_activations=default_scheme.input_activations)
    # M1: config groups nested under an unrelated key
    for k in list(args):
        if _looks_like_groups(args[k]):
            log.warning("recipe key %r holds config groups; treating it as config_groups (quirk M1)", k)
            for gk, g in args.pop(k).items():
                groups[gk] = _scheme_from_group(gk, g)
    if not groups and default_scheme is not None:
        groups["group_0"] = default_scheme
    return groups


_OUT_OF_SCOPE = {"GPTQModifier", "AutoRoundModifier", "SmoothQuantModifier", "SparseGPTModifier"}


def _make_modifier(name: str, args: Dict[str, Any], default_scheme=None):
    args = dict(args or {})
    if name in _OUT_OF_SCOPE:
        raise NotImplementedError(f"{name} is outside this framework's scope (AWQ / RTN quantize path only)")
    ignore = _targets(args.pop("ignore", None))
    groups = _schemes(args, default_scheme)
    if name == "QuantizationModifier":
        args.pop("kv_cache_scheme", None)
        _drop_known(args, ("offload_device",))
        if args:
            raise ValueError(f"QuantizationModifier: unknown arguments {sorted(args)}")
        return QuantizationModifier(config_groups=groups, ignore=ignore)
    if name == "AWQModifier":
        maps = args.pop("mappings", None)
        mappings = None
        if maps:
            mappings = [AWQMapping(smooth_layer=_clean_target(m["smooth_layer"]),
                                   balance_layers=_targets(m["balance_layers"])) for m in maps]
        duo = bool(args.pop("duo_scaling", True))
        n_grid = int(args.pop("n_grid", 20))
        _drop_known(args, ("offload_device", "max_chunk_memory", "sequential_targets"))
        if args:
            raise ValueError(f"AWQModifier: unknown arguments {sorted(args)}")
        return AWQModifier(config_groups=groups, ignore=ignore, mappings=mappings, duo_scaling=duo, n_grid=n_grid)
    raise ValueError(f"unknown modifier {name!r}")


def _drop_known(args, keys):
    for k in keys:
        args.pop(k, None)


def parse_recipe(recipe: Union[str, Dict[str, Any], List[Any]]) -> List[QuantizationModifier]:
    """Recipe path / YAML text / dict / list of modifiers -> ordered modifier list."""
    if isinstance(recipe, (QuantizationModifier,)):
        return [recipe]
    if isinstance(recipe, list) and all(isinstance(m, QuantizationModifier) for m in recipe):
        return list(recipe)
    if isinstance(recipe, str):
        text = open(recipe).read() if os.path.exists(recipe) else recipe
        data = yaml.safe_load(text)
    else:
        data = recipe
    if not isinstance(data, dict):
        raise ValueError("recipe must be a mapping")
    default_scheme = None
    qs = data.get("quantization_scheme")
    if qs is not None:  # M2 shape
        if isinstance(qs, dict) and "type" in qs:
            default_scheme = preset_scheme(qs["type"], _targets(qs.get("targets", ["Linear"])))
    mods: List[QuantizationModifier] = []
    if "modifiers" in data:  # M2 list shape
        for m in data["modifiers"]:
            m = dict(m)
            mods.append(_make_modifier(m.pop("name"), m, default_scheme))
        return mods
    for stage_key, stage in data.items():
        if stage_key in ("quantization_scheme", "version", "metadata") or not isinstance(stage, dict):
            continue
        for group_key, group in stage.items():
            if not isinstance(group, dict):
                continue
            for mod_name, mod_args in group.items():
                mods.append(_make_modifier(mod_name, mod_args, default_scheme))
    if not mods:
        raise ValueError("recipe defines no modifiers")
    return mods


# --------------------------------------------------------------------- target matching
def is_match(name: str, module_type: str, target: str) -> bool:
    """compressed-tensors target semantics: class name, ``re:`` regex (re.match), or exact name."""
    if target.startswith("re:"):
        return re.match(target[3:], name) is not None
    return target == module_type or target == name


def match_any(name: str, module_type: str, targets: List[str]) -> bool:
    return any(is_match(name, module_type, t) for t in targets)


def match_precedence(name: str, module_type: str, target: str) -> Optional[int]:
    """compressed-tensors' precedence among the targets a module matches: exact name (0) over
    ``re:`` regex (1) over class name (2); ``None`` when the target does not match."""
    if target.startswith("re:"):
        return 1 if re.match(target[3:], name) is not None else None
    if target == name:
        return 0
    if target == module_type:
        return 2
    return None
