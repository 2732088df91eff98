"""CRD types (``amd.com/v1`` ClusterPolicy) and the declarative schema machinery."""
