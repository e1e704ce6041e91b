"""Job-name validation (reference: util/validate.go:8-30).

A job name is a DNS-1123 label: <= 63 characters of [a-z0-9-], starting and ending alphanumeric.
(Quirk Q13 fixed: the error message states the real limit, 63.)
"""
import re

DNS1123_LABEL_MAX_LENGTH = 63
_LABEL = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$")


class ValidationError(ValueError):
    pass


def validate_job_name(value: str) -> None:
    if len(value) > DNS1123_LABEL_MAX_LENGTH:
        raise ValidationError(
            f"The len of name {len(value)} is too long, it should be less than "
            f"{DNS1123_LABEL_MAX_LENGTH}")
    if not _LABEL.match(value):
        raise ValidationError(
            "The job name must consist of lower case alphanumeric characters, '-' or '.', and "
            "must start and end with an alphanumeric character.")
