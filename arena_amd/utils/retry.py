"""Retry helpers (reference: util/retry.go:11-62). Only retryable errors are retried."""
import time

from .errors import is_retryable
from .logs import get_logger

log = get_logger("retry")


def retry(attempts: int, sleep_s: float, callback):
    err = None
    for i in range(max(attempts, 1)):
        try:
            callback()
            return None
        except Exception as e:  # noqa: BLE001
            err = e
            if not is_retryable(e):
                log.info("Still need to wait for func, err:%s", e)
                raise
        if i >= attempts - 1:
            break
        time.sleep(sleep_s)
        log.info("Retrying after error: %s", err)
    raise RuntimeError(f"After {attempts} attempts, last error: {err}")


def retry_during(duration_s: float, sleep_s: float, callback, clock=time.monotonic,
                 sleep=time.sleep):
    start = clock()
    i = 0
    while True:
        i += 1
        try:
            callback()
            log.info("Exit the func successfully.")
            return None
        except Exception as e:  # noqa: BLE001
            if not is_retryable(e):
                log.warning("Unexpected err %s", e)
                raise
            log.info("Still need to wait for func, err:%s", e)
            delta = clock() - start
            if delta > duration_s:
                raise RuntimeError(
                    f"After {i} attempts (during {delta:.1f}s), last error: {e}") from e
        sleep(sleep_s)
