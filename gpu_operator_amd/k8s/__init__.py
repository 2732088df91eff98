"""Kubernetes access: dict-object helpers, the client protocol, fake and REST clients."""
from . import errors, objects  # noqa: F401


def __getattr__(name):
    # the in-memory client is for tests and harnesses: node agents do not pay for importing it
    if name == "FakeClient":
        from .fake import FakeClient
        return FakeClient
    raise AttributeError(name)
