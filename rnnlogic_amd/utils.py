"""Config / seeding / logging helpers, API-compatible with the reference's
src/utils.py (load_config, save_config, set_seed, save_model, load_model,
set_logger).  Configs load into an attribute dict (the reference uses
easydict.EasyDict, utils.py:19-33)."""
import itertools
import json
import logging
import os
import random

import numpy as np
import torch
import yaml


class EasyDict(dict):
    """dict with attribute access, recursively (the subset of easydict the
    entry scripts use: cfg.a.b reads and writes)."""

    def __init__(self, d=None, **kw):
        super(EasyDict, self).__init__()
        for k, v in dict(d or {}, **kw).items():
            self[k] = v

    @staticmethod
    def _wrap(v):
        if isinstance(v, dict) and not isinstance(v, EasyDict):
            return EasyDict(v)
        if isinstance(v, (list, tuple)):
            return type(v)(EasyDict._wrap(x) for x in v)
        return v

    def __setitem__(self, k, v):
        super(EasyDict, self).__setitem__(k, self._wrap(v))

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)

    def __setattr__(self, k, v):
        self[k] = v


def _meshgrid(grid):
    keys = list(grid)
    for values in itertools.product(*[grid[k] if isinstance(grid[k], list) else [grid[k]] for k in keys]):
        yield dict(zip(keys, values))


def load_config(cfg_file):
    """utils.py:13-33: one config, or a hyper-parameter grid (`grid --- template`)."""
    with open(cfg_file, "r") as fin:
        raw_text = fin.read()
    if "---" in raw_text:
        import jinja2  # only grid configs need it (reference utils.py:22)
        grid, template = raw_text.split("---")
        grid = yaml.safe_load(grid)
        template = jinja2.Template(template)
        return [EasyDict(yaml.safe_load(template.render(h))) for h in _meshgrid(grid)]
    return [EasyDict(yaml.safe_load(raw_text))]


def save_config(cfg, path):
    with open(os.path.join(path, "config.yaml"), "w") as fo:
        yaml.dump(json.loads(json.dumps(cfg)), fo)


def set_seed(seed):
    """utils.py:39-43: the same four generators, in the same order."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)
    torch.cuda.manual_seed(seed)


def save_model(model, optim, args):
    with open(os.path.join(args.save_path, "config.json"), "w") as fjson:
        json.dump(vars(args), fjson)
    torch.save({"model": model.state_dict(), "optim": optim.state_dict()}, os.path.join(args.save_path, "checkpoint"))


def load_model(model, optim, args):
    checkpoint = torch.load(args.load_path, weights_only=True)
    model.load_state_dict(checkpoint["model"])
    optim.load_state_dict(checkpoint["optim"])


def set_logger(save_path):
    """utils.py:58-69: INFO to save_path/run.log and the console."""
    logging.basicConfig(format="%(asctime)s %(levelname)-8s %(message)s", level=logging.INFO,
                        datefmt="%Y-%m-%d %H:%M:%S", filename=os.path.join(save_path, "run.log"), filemode="w")
    console = logging.StreamHandler()
    console.setLevel(logging.INFO)
    console.setFormatter(logging.Formatter("%(asctime)s %(levelname)-8s %(message)s"))
    logging.getLogger("").addHandler(console)
