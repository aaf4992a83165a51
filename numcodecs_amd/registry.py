"""Codec registry (reference: src/numcodecs/registry.py:10-74).

Same behaviour as numcodecs: ``get_codec(config)`` copies the config, pops
``'id'``, looks the id up in :data:`codec_registry`, then in the
``numcodecs.codecs`` entry-point group (so third-party numcodecs plugins
resolve here too), and raises :class:`UnknownCodecError` otherwise;
``register_codec(cls, codec_id=None)`` replaces any previous registration.
"""

import logging
from importlib.metadata import entry_points

from .errors import UnknownCodecError

__all__ = ["codec_registry", "get_codec", "register_codec", "run_entrypoints"]

logger = logging.getLogger("numcodecs_amd")
codec_registry: dict = {}
entries: dict = {}

ENTRY_POINT_GROUP = "numcodecs.codecs"


def run_entrypoints():
    """(Re)scan the installed entry points of the numcodecs plugin group."""
    entries.clear()
    entries.update({e.name: e for e in entry_points().select(group=ENTRY_POINT_GROUP)})


run_entrypoints()


def get_codec(config):
    """Instantiate the codec described by `config` (not modified)."""
    config = dict(config)
    codec_id = config.pop("id", None)
    cls = codec_registry.get(codec_id)
    if cls is None and codec_id in entries:
        logger.debug("Auto loading codec '%s' from entrypoint", codec_id)
        cls = entries[codec_id].load()
        register_codec(cls, codec_id=codec_id)
    if cls is None:
        raise UnknownCodecError(f"{codec_id!r}")
    return cls.from_config(config)


def register_codec(cls, codec_id=None):
    """Register `cls` under `codec_id` (default ``cls.codec_id``), replacing."""
    if codec_id is None:
        codec_id = cls.codec_id
    logger.debug("Registering codec '%s'", codec_id)
    codec_registry[codec_id] = cls
