"""Exceptions of the codec boundary (reference: src/numcodecs/errors.py:6-26)."""

__all__ = ["UnknownCodecError"]


class UnknownCodecError(ValueError):
    """Raised by :func:`numcodecs_amd.get_codec` for an id nobody registered.

    Same class hierarchy and message as ``numcodecs.errors.UnknownCodecError``
    (a ``ValueError`` whose text is ``codec not available: '<id>'``).
    """

    def __init__(self, codec_id):
        self.codec_id = codec_id
        super().__init__(f"codec not available: '{codec_id}'")
