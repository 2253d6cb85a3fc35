"""Model families: the reference ``Net`` (Linear 784->10) and the north-star ``CNN``."""
from .reference import CNN, MODULES, Net, functional_forward
from .specs import ModelSpec, ParamSpec, cnn_spec, get_spec, linear_spec

__all__ = ["Net", "CNN", "MODULES", "functional_forward", "ModelSpec", "ParamSpec",
           "get_spec", "linear_spec", "cnn_spec"]
