"""The Codec interface (reference: src/numcodecs/abc.py:34-126).

``numcodecs_amd`` codecs are drop-in replacements for numcodecs codecs: same
``codec_id``, same constructor arguments, same ``get_config()`` dicts,
``from_config``, equality-by-config and ``repr``.  ``encode``/``decode``
accept everything the reference accepts (numpy arrays and any object that
exports the buffer protocol) and additionally PyTorch tensors resident on a
HIP device; device tensors come back as device tensors, host buffers as numpy
arrays / bytes exactly as the reference returns them.  The work itself always
runs on the GPU (libmcodec.so); there is no CPU path.
"""

from abc import ABC, abstractmethod

__all__ = ["Codec"]


class Codec(ABC):
    """Codec abstract base class."""

    #: codec identifier, the ``'id'`` of the config dict (override in sub-class)
    codec_id: "str | None" = None

    @abstractmethod
    def encode(self, buf):  # pragma: no cover
        """Encode data in `buf` (buffer-like or device tensor)."""

    @abstractmethod
    def decode(self, buf, out=None):  # pragma: no cover
        """Decode data in `buf`; `out`, if given, must be exactly the right size."""

    def get_config(self):
        """JSON-serialisable configuration; every public attribute plus 'id'."""
        config = {"id": self.codec_id}
        config.update((k, v) for k, v in self.__dict__.items() if not k.startswith("_"))
        return config

    @classmethod
    def from_config(cls, config):
        """Instantiate from a config dict whose 'id' has already been removed."""
        return cls(**config)

    def __eq__(self, other):
        try:
            return self.get_config() == other.get_config()
        except AttributeError:
            return False

    def __repr__(self):
        params = ", ".join(
            f"{k}={getattr(self, k)!r}" for k in sorted(self.__dict__) if not k.startswith("_")
        )
        return f"{type(self).__name__}({params})"
