"""gpu_operator_amd — an MI355X-native Kubernetes GPU operator.

Control plane (ClusterPolicy reconciler, state manager, upgrade FSM), node agents (validator,
device plugin, node labeller, partition manager, metrics exporter, CDI runtime hook) and the
validator's native GPU workloads (CDNA4 MFMA GEMM, RCCL all-reduce). See README.md.
"""

__version__ = "0.1.0"
