"""bioimitation — MI355X-native vectorized env.step() for bioimitation-gym.

Drop-in surface: the reference's env IDs (bioimitation/__init__.py:23-143 of
UtkarshMishra04/bioimitation-gym), ``Env(config)`` classes with
``reset()/step()``, plus :class:`VectorEnv` for batched GPU stepping.
"""
from .registry import REGISTERED_IDS, RECIPES, env_spec, load_pack  # noqa: F401

__all__ = ['REGISTERED_IDS', 'RECIPES', 'env_spec', 'load_pack', 'VectorEnv', 'MixedVectorEnv', 'make',
           'RLlibVectorEnv', 'GymVectorEnv', 'MeanStdFilter']

_LAZY = {'VectorEnv': 'vector_env', 'MixedVectorEnv': 'vector_env', 'make': 'envs', 'RLlibVectorEnv': 'adapters',
         'GymVectorEnv': 'adapters', 'MeanStdFilter': 'adapters'}


def __getattr__(name):
    if name in _LAZY:
        import importlib
        return getattr(importlib.import_module('.' + _LAZY[name], __name__), name)
    raise AttributeError(name)
