"""API errors with the HTTP semantics of the Kubernetes API server."""

from __future__ import annotations


class ApiError(Exception):
    status = 500
    reason = "InternalError"

    def __init__(self, message: str = "", status: int | None = None, reason: str | None = None):
        super().__init__(message or self.reason)
        if status is not None:
            self.status = status
        if reason is not None:
            self.reason = reason


class NotFound(ApiError):
    status = 404
    reason = "NotFound"


class AlreadyExists(ApiError):
    status = 409
    reason = "AlreadyExists"


class Conflict(ApiError):
    status = 409
    reason = "Conflict"


class Invalid(ApiError):
    status = 422
    reason = "Invalid"


class Forbidden(ApiError):
    status = 403
    reason = "Forbidden"


class TooManyRequests(ApiError):
    """Returned by the eviction subresource when a PodDisruptionBudget blocks eviction."""

    status = 429
    reason = "TooManyRequests"


class NoKindMatch(ApiError):
    """The kind is not served by the API server (e.g. ServiceMonitor without prometheus-operator)."""

    status = 404
    reason = "NoKindMatch"


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.status == 404


def is_conflict(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.status == 409


def from_status(status: int, message: str, reason: str = "") -> ApiError:
    if status == 404:
        return NotFound(message)
    if status == 409:
        return AlreadyExists(message) if reason == "AlreadyExists" else Conflict(message)
    if status == 422:
        return Invalid(message)
    if status == 403:
        return Forbidden(message)
    if status == 429:
        return TooManyRequests(message)
    return ApiError(message, status=status, reason=reason or None)
