"""Attribute-dict config over YAML (lib/config.py:5-81), loaded with SafeLoader.

`cfg_get` reads an optional key from either this Config or the reference's own
Config object, whose __getattr__ raises KeyError rather than AttributeError
(lib/config.py:26-27), so a reference config can be handed to pggan_amd as is."""
import os
import shutil

import yaml


def cfg_get(args, key, default=None):
    try:
        v = getattr(args, key)
    except (AttributeError, KeyError):
        return default
    return default if v is None and default is not None else v


class Config(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = Config(v) if isinstance(v, dict) and not isinstance(v, Config) else v

    @property
    def __dict__(self):
        return self

    @staticmethod
    def from_yaml(path):
        with open(path) as f:
            return Config(yaml.safe_load(f))

    @staticmethod
    def from_dict(d):
        return Config(d)

    @staticmethod
    def get_empty():
        return Config()

    def save_yaml(self, read_path):
        """lib/config.py:15-16: copy the YAML next to the run's results."""
        d = f"{self.get('save_root', 'train_result')}/{self.run_id}"
        os.makedirs(d, exist_ok=True)
        shutil.copy(read_path, f"{d}/config_{self.run_id}.yaml")

    def update(self, other=None, **kw):
        super().update(other or {}, **kw)

    @classmethod
    def extraction_dictionary(cls, config):
        return {k: (cls.extraction_dictionary(v) if isinstance(v, dict) else v)
                for k, v in config.items()}
