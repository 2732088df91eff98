"""Controller runtime: work queue, controllers, leader election, manager (probes/metrics)."""
from .controller import Controller, Result  # noqa: F401
from .manager import Manager  # noqa: F401
from .workqueue import ExponentialBackoff, WorkQueue  # noqa: F401
