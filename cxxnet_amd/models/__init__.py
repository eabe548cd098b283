"""Model zoo: .conf network definitions (AlexNet, GoogLeNet/Inception-v1, VGG-16,
MNIST MLP/conv, Kaggle-bowl convnet) and helpers to load them."""
from __future__ import annotations

import os
from typing import List, Tuple

CONF_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "confs")


def conf_path(name: str) -> str:
    p = os.path.join(CONF_DIR, name if name.endswith(".conf") else name + ".conf")
    if not os.path.exists(p):
        raise FileNotFoundError(f"no model conf named {name} (have: {available()})")
    return p


def available() -> List[str]:
    return sorted(f[:-5] for f in os.listdir(CONF_DIR) if f.endswith(".conf"))


def load_conf(name: str, overrides: List[Tuple[str, str]] = ()) -> List[Tuple[str, str]]:
    from .. import native
    pairs = list(native.rt().parse_config_file(conf_path(name)))
    return pairs + list(overrides)
