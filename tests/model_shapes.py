"""Reference state_dict names/shapes at the benchmark configs (tests/golden/state_dict_keys.json)."""
import json
import os

import torch

_P = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "state_dict_keys.json")


def keys(name):
    with open(_P) as f:
        return json.load(f)[name]


def empty_state_dict(name):
    return {k: torch.zeros(v) for k, v in keys(name).items()}
