"""YAML configuration with `include:` indirection and dotted access.

Same semantics as the reference loader (src/utils/config_utils.py): `DictConfig` attribute access
(:6-14), recursive `include:<path>` unpacking (:20-30), recursive merge where the second config
wins (:36-52, :59-75), string -> typed values for CLI kwargs (:94-118) and dotted-key kwargs ->
nested dict (:123-140).  Pinned by tests/golden/configs.json (produced by the reference loader).
"""
from __future__ import annotations

import copy

import yaml


class DictConfig(dict):
    """dict with attribute access; nested dicts come back as DictConfig."""

    def __getattr__(self, name):
        try:
            v = self[name]
        except KeyError as e:
            raise AttributeError(name) from e
        return DictConfig(v) if isinstance(v, dict) and not isinstance(v, DictConfig) else v

    def get_dict(self):
        return dict(self)


def _load(path):
    with open(path, "r") as f:
        return yaml.safe_load(f)


def _unpack(node):
    if isinstance(node, str) and node.split(":")[0] == "include":
        node = _load(node.split(":", 1)[1])
    if isinstance(node, dict):
        for k in list(node):
            node[k] = _unpack(node[k])
    return node


def _merge(base, override):
    if isinstance(override, dict):
        if not isinstance(base, dict):
            base = {}
        for k in override:
            base[k] = _merge(base.get(k, {}), override[k])
        return base
    return override


def update_config(default_config, config=None) -> DictConfig:
    """Merge `config` over `default_config` (either may be a YAML path); includes are unpacked.

    As in the reference, a non-dict `config` (e.g. an argparse Namespace) contributes nothing."""
    if isinstance(default_config, str):
        default_config = _load(default_config)
    config = default_config if config is None else config
    if isinstance(config, str):
        config = _load(config)
    base = _unpack(copy.deepcopy(default_config) if isinstance(default_config, dict) else default_config)
    over = _unpack(copy.deepcopy(config) if isinstance(config, dict) else config)
    return DictConfig(_merge(base, over))


def convert_to_dtype(value: str):
    value = value.strip()
    if value[:1] == "[" and value[-1:] == "]":
        return [convert_to_dtype(v) for v in value[1:-1].split(",")]
    if value in ("null", "None", "none"):
        return None
    if value in ("true", "True"):
        return True
    if value in ("false", "False"):
        return False
    if value.isdigit() or value.replace("-", "").isdigit():
        return int(value)
    try:
        return float(value)
    except ValueError:
        return value


def config_from_kwargs(kwargs) -> DictConfig:
    out: dict = {}
    for key, value in (kwargs or {}).items():
        value = convert_to_dtype(value)
        cur = out
        parts = key.split(".")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = value
    return DictConfig(out)


def load_run_config(model_yaml: str, train_yaml: str) -> DictConfig:
    """`src/train.py:27-29`: model YAML included under `model`, then merged under the train YAML."""
    cfg = config_from_kwargs({"model": "include:" + model_yaml})
    return update_config(train_yaml, cfg)
