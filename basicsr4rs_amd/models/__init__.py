"""Model registry surface (mirror of basicsr/models/__init__.py:10-29)."""
import importlib
import os
from copy import deepcopy
from os import path as osp

from ..utils.registry import MODEL_REGISTRY

__all__ = ['build_model']

model_folder = osp.dirname(osp.abspath(__file__))
model_filenames = sorted(osp.splitext(f)[0] for f in os.listdir(model_folder) if f.endswith('_model.py'))
_model_modules = [importlib.import_module(f'{__name__}.{name}') for name in model_filenames]


def build_model(opt):
    opt = deepcopy(opt)
    model = MODEL_REGISTRY.get(opt['model_type'])(opt)
    return model
