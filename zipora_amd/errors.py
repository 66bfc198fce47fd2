"""ZiporaError mirror (src/error.rs:10, InvalidData at error.rs:139) for C ABI status codes."""
from . import _lib


class ZiporaError(Exception):
    """Raised for any non-zero C ABI status; .code is the CResult value (src/ffi/mod.rs:29-58)."""

    def __init__(self, code_or_message, message=None):
        if message is None:  # ZiporaError("...") == invalid data / parameter
            code_or_message, message = _lib.ZR_INVALID_INPUT, code_or_message
        super().__init__(message)
        self.code = code_or_message

    @property
    def is_invalid_data(self):
        return self.code == _lib.ZR_INVALID_INPUT


def check(status):
    if status != _lib.ZR_OK:
        raise ZiporaError(status, _lib.last_error() or f"status {status}")
    return status
