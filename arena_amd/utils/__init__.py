"""L0 utilities (reference: util/*.go). Validation, durations, retry, logging, random ids, tables."""
from .duration import parse_duration, short_human_duration  # noqa: F401
from .errors import (ArenaError, is_connection_refused, is_need_wait,  # noqa: F401
                     is_retryable, is_unexpected_eof, NEED_WAIT)
from .logs import get_logger, set_log_level  # noqa: F401
from .random import random_int32  # noqa: F401
from .retry import retry, retry_during  # noqa: F401
from .tabwriter import TabWriter  # noqa: F401
from .validate import validate_job_name  # noqa: F401
from .volume import parse_data_dir_raw, validate_datasets  # noqa: F401
