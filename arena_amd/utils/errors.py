"""Retryable-error classification (reference: util/errors.go:5-22)."""

NEED_WAIT = "Need waited."


class ArenaError(RuntimeError):
    """A user-facing error: the CLI prints it and exits 1."""


def _contains(err, text: str) -> bool:
    return text in str(err)


def is_need_wait(err) -> bool:
    return _contains(err, NEED_WAIT)


def is_connection_refused(err) -> bool:
    return _contains(err, "connection refused")


def is_unexpected_eof(err) -> bool:
    return _contains(err, "unexpected EOF")


def is_retryable(err) -> bool:
    return is_need_wait(err) or is_connection_refused(err) or is_unexpected_eof(err)
