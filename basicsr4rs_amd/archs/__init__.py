"""Arch registry surface (mirror of basicsr/archs/__init__.py:10-24).

Every ``*_arch.py`` module in this package is imported so its classes register in
ARCH_REGISTRY; ``build_network(opt)`` pops ``type`` and builds ``ARCH_REGISTRY.get(type)(**opt)``.
"""
import importlib
from copy import deepcopy
from os import path as osp

from ..utils.registry import ARCH_REGISTRY

__all__ = ['build_network']

arch_folder = osp.dirname(osp.abspath(__file__))
arch_filenames = sorted(osp.splitext(f)[0] for f in __import__('os').listdir(arch_folder) if f.endswith('_arch.py'))
_arch_modules = [importlib.import_module(f'{__name__}.{name}') for name in arch_filenames]


def build_network(opt):
    opt = deepcopy(opt)
    network_type = opt.pop('type')
    net = ARCH_REGISTRY.get(network_type)(**opt)
    return net
