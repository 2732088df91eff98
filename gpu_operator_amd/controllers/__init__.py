"""ClusterPolicy reconciler, state manager, operand transforms and the driver-upgrade FSM."""
