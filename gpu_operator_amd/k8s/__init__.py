"""Kubernetes access: dict-object helpers, the client protocol, fake and REST clients."""
from . import errors, objects  # noqa: F401
from .fake import FakeClient  # noqa: F401
