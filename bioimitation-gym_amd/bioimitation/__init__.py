"""bioimitation — MI355X-native vectorized env.step() for bioimitation-gym.

Drop-in surface: the reference's env IDs (bioimitation/__init__.py:23-143 of
UtkarshMishra04/bioimitation-gym), ``Env(config)`` classes with
``reset()/step()``, plus :class:`VectorEnv` for batched GPU stepping.
"""
from .registry import REGISTERED_IDS, RECIPES, env_spec, load_pack  # noqa: F401

__all__ = ['REGISTERED_IDS', 'RECIPES', 'env_spec', 'load_pack', 'VectorEnv', 'make']


def __getattr__(name):
    if name == 'VectorEnv':
        from .vector_env import VectorEnv
        return VectorEnv
    if name == 'make':
        from .envs import make
        return make
    raise AttributeError(name)
