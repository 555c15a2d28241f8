"""Name -> class registry with Dassl semantics (Dassl.pytorch/dassl/utils/registry.py:36-68,
dassl/engine/build.py:3-11): duplicate names raise KeyError, unknown names raise KeyError
listing the registered ones; ``cfg.TRAINER.NAME`` selects the trainer class."""


class Registry:
    def __init__(self, name):
        self._name = name
        self._obj_map = {}

    def _do_register(self, name, obj, force=False):
        if name in self._obj_map and not force:
            raise KeyError(f'An object named "{name}" was already registered in "{self._name}" registry')
        self._obj_map[name] = obj

    def register(self, obj=None, force=False):
        if obj is None:
            def deco(o):
                self._do_register(o.__name__, o, force=force)
                return o
            return deco
        self._do_register(obj.__name__, obj, force=force)
        return obj

    def get(self, name):
        if name not in self._obj_map:
            raise KeyError(f'Object name "{name}" does not exist in "{self._name}" registry; '
                           f"available: {self.registered_names()}")
        return self._obj_map[name]

    def registered_names(self):
        return list(self._obj_map.keys())


TRAINER_REGISTRY = Registry("TRAINER")


def build_trainer(cfg, **kwargs):
    """dassl/engine/build.py:6-11 analogue."""
    from .. import trainers  # noqa: F401  (registers CoOp / CoCoOp)
    return TRAINER_REGISTRY.get(cfg.TRAINER.NAME)(cfg, **kwargs)
