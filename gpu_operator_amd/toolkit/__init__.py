"""AMD container toolkit: CDI spec generator, runtime configuration and the install daemon
(``amd-ctk``); the OCI runtime shim itself is native (native/toolkit/amd_container_runtime.cpp)."""
