from .clusterpolicy import *  # noqa: F401,F403
from .clusterpolicy import ClusterPolicy, ClusterPolicySpec, image_path  # noqa: F401
