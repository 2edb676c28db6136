"""Name -> object registries: the drop-in surface of basicsr/utils/registry.py:4-88.

Same contract as the reference: ``register(obj=None, suffix=None)`` works as a decorator
or a call and keys objects by ``__name__`` (+ ``_suffix``); registering a name twice
asserts; ``get(name, suffix='basicsr')`` falls back to ``name_suffix`` and raises KeyError
when neither exists.
"""


class Registry:

    def __init__(self, name):
        self._name = name
        self._obj_map = {}

    def _do_register(self, name, obj, suffix=None):
        if isinstance(suffix, str):
            name = f'{name}_{suffix}'
        assert name not in self._obj_map, f"An object named '{name}' was already registered in '{self._name}' registry!"
        self._obj_map[name] = obj

    def register(self, obj=None, suffix=None):
        if obj is None:

            def deco(func_or_class):
                self._do_register(func_or_class.__name__, func_or_class, suffix)
                return func_or_class

            return deco
        self._do_register(obj.__name__, obj, suffix)

    def get(self, name, suffix='basicsr'):
        ret = self._obj_map.get(name)
        if ret is None:
            ret = self._obj_map.get(f'{name}_{suffix}')
            print(f'Name {name} is not found, use name: {name}_{suffix}!')
        if ret is None:
            raise KeyError(f"No object named '{name}' found in '{self._name}' registry!")
        return ret

    def __contains__(self, name):
        return name in self._obj_map

    def __iter__(self):
        return iter(self._obj_map.items())

    def keys(self):
        return self._obj_map.keys()


DATASET_REGISTRY = Registry('dataset')
ARCH_REGISTRY = Registry('arch')
MODEL_REGISTRY = Registry('model')
LOSS_REGISTRY = Registry('loss')
METRIC_REGISTRY = Registry('metric')
