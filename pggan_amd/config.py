"""Attribute-dict config over YAML (lib/config.py:5-81), loaded with SafeLoader."""
import yaml


class Config(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @property
    def __dict__(self):
        return self

    @staticmethod
    def from_yaml(path):
        with open(path) as f:
            return Config(yaml.safe_load(f))

    def update(self, other=None, **kw):
        super().update(other or {}, **kw)
