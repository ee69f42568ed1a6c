"""Configuration system.

Two front-ends over one mechanism:

* ``CfgNode`` — the upstream-minGPT style attribute bag with ``merge_from_dict`` and
  ``merge_from_args(["--trainer.batch_size=32", ...])`` (advertised by the reference at
  ``/root/reference/README.md:27-54``).
* ``load_run_config(path, overrides)`` — reads the reference's four-section YAML
  (``gpt_config`` / ``optimizer_config`` / ``data_config`` / ``trainer_config``,
  ``/root/reference/mingpt/gpt2_config.yaml:1-18``) into the four typed dataclasses that
  ``/root/reference/mingpt/train.py:36-39`` splats them into.  Hydra is not installed, so
  Hydra-style ``section.key=value`` overrides and CfgNode-style ``--section.key=value``
  overrides are both parsed here.  The reference's YAML key typo ``n_embd``
  (defect D14) is accepted as an alias of ``n_embed``.
"""
from __future__ import annotations

import ast
import dataclasses
import json
from typing import Any, Dict, Iterable, List, Optional

import yaml


class CfgNode:
    """A lightweight configuration class inspired by yacs (upstream minGPT API)."""

    def __init__(self, **kwargs):
        self.__dict__.update(kwargs)

    def __str__(self):
        return self._str_helper(0)

    def _str_helper(self, indent):
        parts = []
        for k, v in self.__dict__.items():
            if isinstance(v, CfgNode):
                parts.append("%s:\n" % k)
                parts.append(v._str_helper(indent + 1))
            else:
                parts.append("%s: %s\n" % (k, v))
        return "".join(" " * (indent * 4) + p for p in parts)

    def to_dict(self) -> Dict[str, Any]:
        return {k: v.to_dict() if isinstance(v, CfgNode) else v for k, v in self.__dict__.items()}

    def merge_from_dict(self, d: Dict[str, Any]) -> None:
        for k, v in d.items():
            if isinstance(v, dict) and isinstance(getattr(self, k, None), CfgNode):
                getattr(self, k).merge_from_dict(v)
            else:
                setattr(self, k, v)

    def merge_from_args(self, args: Iterable[str]) -> None:
        """Apply ``--a.b.c=value`` (or ``a.b.c=value``) overrides.

        Values are parsed as Python literals when possible, else kept as strings.
        Unknown leaf keys raise, which catches typos early.
        """
        for arg in args:
            key, val = _split_override(arg)
            keys = key.split(".")
            obj = self
            for k in keys[:-1]:
                obj = getattr(obj, k)
            leaf = keys[-1]
            assert hasattr(obj, leaf), f"{key} is not an attribute that exists in the config"
            setattr(obj, leaf, _parse_value(val))


def _split_override(arg: str):
    if "=" not in arg:
        raise ValueError(f"override {arg!r} must look like key=value")
    key, val = arg.split("=", 1)
    key = key.lstrip("-").lstrip("+")
    return key, val


def _parse_value(val: str) -> Any:
    try:
        return ast.literal_eval(val)
    except (ValueError, SyntaxError):
        low = val.lower()
        if low in ("true", "false"):
            return low == "true"
        if low in ("none", "null"):
            return None
        return val


# Aliases for YAML keys, applied per section before building the dataclass.
_KEY_ALIASES = {
    "gpt_config": {"n_embd": "n_embed", "embd_pdrop": "embed_drop", "resid_pdrop": "resid_drop",
                   "attn_pdrop": "attn_drop"},
    "optimizer_config": {"lr": "learning_rate"},
    "data_config": {},
    "trainer_config": {},
}


def _coerce(dc_type, section: str, values: Dict[str, Any]):
    aliases = _KEY_ALIASES.get(section, {})
    fields = {f.name: f for f in dataclasses.fields(dc_type)}
    kwargs = {}
    for k, v in (values or {}).items():
        k = aliases.get(k, k)
        if k not in fields:
            raise KeyError(f"unknown key {k!r} in section {section!r} (valid: {sorted(fields)})")
        if k == "betas" and isinstance(v, list):
            v = tuple(v)
        kwargs[k] = v
    return dc_type(**kwargs)


def load_yaml(path: str) -> Dict[str, Any]:
    import fsspec

    with fsspec.open(path, "r") as f:
        return yaml.safe_load(f) or {}


def apply_overrides(raw: Dict[str, Any], overrides: Optional[List[str]]) -> Dict[str, Any]:
    raw = json.loads(json.dumps(raw))  # deep copy of plain data
    for arg in overrides or []:
        key, val = _split_override(arg)
        keys = key.split(".")
        node = raw
        for k in keys[:-1]:
            node = node.setdefault(k, {})
        node[keys[-1]] = _parse_value(val)
    return raw


@dataclasses.dataclass
class RunConfig:
    gpt_config: Any
    optimizer_config: Any
    data_config: Any
    trainer_config: Any


def load_run_config(path: Optional[str] = None, overrides: Optional[List[str]] = None,
                    raw: Optional[Dict[str, Any]] = None) -> RunConfig:
    """Load the reference-shaped four-section YAML into typed dataclasses."""
    from ..models.config import GPTConfig, OptimizerConfig
    from ..data.char_dataset import DataConfig
    from ..trainer import GPTTrainerConfig

    if raw is None:
        raw = load_yaml(path) if path else {}
    raw = {k: v for k, v in raw.items() if k != "hydra"}  # hydra's run-dir section is not ours
    raw = apply_overrides(raw, overrides)
    return RunConfig(
        gpt_config=_coerce(GPTConfig, "gpt_config", raw.get("gpt_config")),
        optimizer_config=_coerce(OptimizerConfig, "optimizer_config", raw.get("optimizer_config")),
        data_config=_coerce(DataConfig, "data_config", raw.get("data_config")),
        trainer_config=_coerce(GPTTrainerConfig, "trainer_config", raw.get("trainer_config")),
    )
