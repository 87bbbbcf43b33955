"""Run configuration: the reference's 3-level YAML (run config -> recipe path + calibration set),
same keys and path resolution as src/quantizers/config.py:52-114 and scripts/do_oneshot.py:111-135.
The calibration-set file is parsed and validated as the reference does
(CalibrationSetConfig.from_file, src/quantizers/calibration_sets.py:208-247); its *content*
comes from the reference-format parquet cache (calibration.py) -- building it from Hub datasets
is network-bound and out of scope -- or from a local tokenized file / synthetic ids (cli.py)."""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, Optional

import logging

import yaml


@dataclass
class ModelConfig:
    name: str
    revision: str = "main"


@dataclass
class RunConfig:
    model: ModelConfig
    recipe: str
    calibration_set: Optional[str] = None
    calibration: Optional[Dict[str, Any]] = None
    config_path: Optional[str] = None

    def resolve_recipe(self) -> str:
        """scripts/do_oneshot.py:124-135: relative to the config dir, then <dir>/recipes/."""
        p = self.recipe
        if not Path(p).is_absolute() and self.config_path:
            cand = Path(self.config_path).parent / p
            if not cand.exists():
                cand = Path(self.config_path).parent / "recipes" / p
            p = str(cand)
        if not Path(p).exists():
            raise ValueError(f"Recipe file not found: {p}")
        return p

    def output_dir(self) -> str:
        """scripts/do_oneshot.py:114-121: outputs/<model basename>-<recipe stem without recipe_>."""
        name = self.model.name.split("/")[-1] if "/" in self.model.name else self.model.name
        return f"outputs/{name}-{Path(self.recipe).stem.replace('recipe_', '')}"


def load_run_config(path: str) -> RunConfig:
    p = Path(path)
    if not p.exists():
        raise ValueError(f"Config file not found: {path}")
    data = yaml.safe_load(p.read_text()) or {}
    m = data.get("model", {}) or {}
    if not m.get("name"):
        raise ValueError("Model name is required")
    q = data.get("quantization", {}) or {}
    if not q.get("recipe"):
        raise ValueError("Recipe path is required")
    calib = q.get("calibration_set") or data.get("calibration_set")
    calib_cfg = None
    if calib:
        cp = calib if calib.endswith(".yaml") else calib + ".yaml"
        if not Path(cp).is_absolute():
            base = p.parent
            cp = str(base / cp[len("configs/"):]) if cp.startswith("configs/") else str(base / cp)
        if Path(cp).exists():
            from .calibration import normalise
            calib_cfg = normalise(yaml.safe_load(Path(cp).read_text()) or {})
        else:  # the reference raises here; offline runs may still pass --calib-file / --calib-random
            logging.getLogger(__name__).warning("Calibration set not found: %s", cp)
        calib = cp
    return RunConfig(model=ModelConfig(m["name"], m.get("revision", "main")), recipe=q["recipe"],
                     calibration_set=calib, calibration=calib_cfg, config_path=str(p))
