"""kubelet gRPC APIs used by the node agents, built from descriptors at import time:

* ``v1beta1`` device plugin API (Registration + DevicePlugin services) — the contract the
  ROCm device plugin and the sandbox (KubeVirt) device plugin serve;
* ``v1`` pod-resources API (PodResourcesLister) — how the metrics exporter attributes GPUs
  to pods.

Field names and numbers follow the upstream Kubernetes .proto files, so the wire format is
the kubelet's. Messages are created through ``descriptor_pb2`` + ``message_factory`` (no
protoc/grpc_tools step in the build).
"""

from __future__ import annotations

from typing import Dict, List, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

T = descriptor_pb2.FieldDescriptorProto
STRING, BOOL, INT64, INT32, MSG = T.TYPE_STRING, T.TYPE_BOOL, T.TYPE_INT64, T.TYPE_INT32, T.TYPE_MESSAGE
OPT, REP = T.LABEL_OPTIONAL, T.LABEL_REPEATED

# message -> [(field, number, type, label, message type or None)]
DEVICEPLUGIN_MESSAGES: Dict[str, List[Tuple]] = {
    "DevicePluginOptions": [("pre_start_required", 1, BOOL, OPT, None),
                            ("get_preferred_allocation_available", 2, BOOL, OPT, None)],
    "RegisterRequest": [("version", 1, STRING, OPT, None), ("endpoint", 2, STRING, OPT, None),
                        ("resource_name", 3, STRING, OPT, None),
                        ("options", 4, MSG, OPT, "DevicePluginOptions")],
    "Empty": [],
    "ListAndWatchResponse": [("devices", 1, MSG, REP, "Device")],
    "TopologyInfo": [("nodes", 1, MSG, REP, "NUMANode")],
    "NUMANode": [("ID", 1, INT64, OPT, None)],
    "Device": [("ID", 1, STRING, OPT, None), ("health", 2, STRING, OPT, None),
               ("topology", 3, MSG, OPT, "TopologyInfo")],
    "PreStartContainerRequest": [("devicesIDs", 1, STRING, REP, None)],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, MSG, REP, "ContainerPreferredAllocationRequest")],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, STRING, REP, None),
                                            ("must_include_deviceIDs", 2, STRING, REP, None),
                                            ("allocation_size", 3, INT32, OPT, None)],
    "PreferredAllocationResponse": [("container_responses", 1, MSG, REP, "ContainerPreferredAllocationResponse")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, STRING, REP, None)],
    "AllocateRequest": [("container_requests", 1, MSG, REP, "ContainerAllocateRequest")],
    "ContainerAllocateRequest": [("devicesIDs", 1, STRING, REP, None)],
    "CDIDevice": [("name", 1, STRING, OPT, None)],
    "AllocateResponse": [("container_responses", 1, MSG, REP, "ContainerAllocateResponse")],
    "ContainerAllocateResponse": [("envs", 1, "map", REP, None), ("mounts", 2, MSG, REP, "Mount"),
                                  ("devices", 3, MSG, REP, "DeviceSpec"), ("annotations", 4, "map", REP, None),
                                  ("cdi_devices", 5, MSG, REP, "CDIDevice")],
    "Mount": [("container_path", 1, STRING, OPT, None), ("host_path", 2, STRING, OPT, None),
              ("read_only", 3, BOOL, OPT, None)],
    "DeviceSpec": [("container_path", 1, STRING, OPT, None), ("host_path", 2, STRING, OPT, None),
                   ("permissions", 3, STRING, OPT, None)],
}

PODRESOURCES_MESSAGES: Dict[str, List[Tuple]] = {
    "ListPodResourcesRequest": [],
    "ListPodResourcesResponse": [("pod_resources", 1, MSG, REP, "PodResources")],
    "PodResources": [("name", 1, STRING, OPT, None), ("namespace", 2, STRING, OPT, None),
                     ("containers", 3, MSG, REP, "ContainerResources")],
    "ContainerResources": [("name", 1, STRING, OPT, None), ("devices", 2, MSG, REP, "ContainerDevices"),
                           ("cpu_ids", 3, INT64, REP, None)],
    "ContainerDevices": [("resource_name", 1, STRING, OPT, None), ("device_ids", 2, STRING, REP, None),
                         ("topology", 3, MSG, OPT, "TopologyInfo")],
    "TopologyInfo": [("nodes", 1, MSG, REP, "NUMANode")],
    "NUMANode": [("ID", 1, INT64, OPT, None)],
}


def _build(package: str, fname: str, messages: Dict[str, List[Tuple]]):
    fdp = descriptor_pb2.FileDescriptorProto(name=fname, package=package, syntax="proto3")
    for mname, fields in messages.items():
        m = fdp.message_type.add(name=mname)
        for fname_, num, typ, label, mtype in fields:
            f = m.field.add(name=fname_, number=num, label=label)
            if typ == "map":
                entry = m.nested_type.add(name="".join(p.capitalize() for p in fname_.split("_")) + "Entry")
                entry.options.map_entry = True
                entry.field.add(name="key", number=1, type=STRING, label=OPT)
                entry.field.add(name="value", number=2, type=STRING, label=OPT)
                f.type = MSG
                f.type_name = f".{package}.{mname}.{entry.name}"
            else:
                f.type = typ
                if mtype:
                    f.type_name = f".{package}.{mtype}"
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    out = {}
    for mname in messages:
        desc = pool.FindMessageTypeByName(f"{package}.{mname}")
        out[mname] = message_factory.GetMessageClass(desc)
    return out


DP = _build("v1beta1", "deviceplugin_v1beta1.proto", DEVICEPLUGIN_MESSAGES)
PR = _build("v1", "podresources_v1.proto", PODRESOURCES_MESSAGES)

API_VERSION = "v1beta1"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
KUBELET_SOCKET = DEVICE_PLUGIN_PATH + "kubelet.sock"
POD_RESOURCES_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
HEALTHY, UNHEALTHY = "Healthy", "Unhealthy"


def _m(name: str, pkg: str = "dp"):
    return (DP if pkg == "dp" else PR)[name]


def registration_stub(channel):
    """Client for kubelet's Registration service."""
    return channel.unary_unary("/v1beta1.Registration/Register",
                               request_serializer=_m("RegisterRequest").SerializeToString,
                               response_deserializer=_m("Empty").FromString)


def device_plugin_handler(servicer):
    """gRPC generic handler serving ``servicer`` as v1beta1.DevicePlugin."""
    import grpc
    u = grpc.unary_unary_rpc_method_handler
    s = grpc.unary_stream_rpc_method_handler
    return grpc.method_handlers_generic_handler("v1beta1.DevicePlugin", {
        "GetDevicePluginOptions": u(servicer.GetDevicePluginOptions, _m("Empty").FromString,
                                    _m("DevicePluginOptions").SerializeToString),
        "ListAndWatch": s(servicer.ListAndWatch, _m("Empty").FromString,
                          _m("ListAndWatchResponse").SerializeToString),
        "GetPreferredAllocation": u(servicer.GetPreferredAllocation, _m("PreferredAllocationRequest").FromString,
                                    _m("PreferredAllocationResponse").SerializeToString),
        "Allocate": u(servicer.Allocate, _m("AllocateRequest").FromString, _m("AllocateResponse").SerializeToString),
        "PreStartContainer": u(servicer.PreStartContainer, _m("PreStartContainerRequest").FromString,
                               _m("PreStartContainerResponse").SerializeToString),
    })


def device_plugin_stub(channel):
    """Client side of a device plugin (what kubelet calls) — used by tests and tools."""
    return {
        "GetDevicePluginOptions": channel.unary_unary("/v1beta1.DevicePlugin/GetDevicePluginOptions",
                                                      _m("Empty").SerializeToString,
                                                      _m("DevicePluginOptions").FromString),
        "ListAndWatch": channel.unary_stream("/v1beta1.DevicePlugin/ListAndWatch", _m("Empty").SerializeToString,
                                             _m("ListAndWatchResponse").FromString),
        "GetPreferredAllocation": channel.unary_unary("/v1beta1.DevicePlugin/GetPreferredAllocation",
                                                      _m("PreferredAllocationRequest").SerializeToString,
                                                      _m("PreferredAllocationResponse").FromString),
        "Allocate": channel.unary_unary("/v1beta1.DevicePlugin/Allocate", _m("AllocateRequest").SerializeToString,
                                        _m("AllocateResponse").FromString),
        "PreStartContainer": channel.unary_unary("/v1beta1.DevicePlugin/PreStartContainer",
                                                 _m("PreStartContainerRequest").SerializeToString,
                                                 _m("PreStartContainerResponse").FromString),
    }


def registration_handler(on_register):
    """Server side of kubelet's Registration service (tests play kubelet)."""
    import grpc

    def register(req, ctx):
        on_register(req)
        return _m("Empty")()
    return grpc.method_handlers_generic_handler("v1beta1.Registration", {
        "Register": grpc.unary_unary_rpc_method_handler(register, _m("RegisterRequest").FromString,
                                                        _m("Empty").SerializeToString)})


def pod_resources_stub(channel):
    return channel.unary_unary("/v1.PodResourcesLister/List",
                               request_serializer=_m("ListPodResourcesRequest", "pr").SerializeToString,
                               response_deserializer=_m("ListPodResourcesResponse", "pr").FromString)


def pod_resources_handler(list_fn):
    import grpc
    return grpc.method_handlers_generic_handler("v1.PodResourcesLister", {
        "List": grpc.unary_unary_rpc_method_handler(list_fn, _m("ListPodResourcesRequest", "pr").FromString,
                                                    _m("ListPodResourcesResponse", "pr").SerializeToString)})
