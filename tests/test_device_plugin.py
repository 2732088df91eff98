"""ROCm device plugin: discovery/naming, kubelet registration, ListAndWatch, Allocate and
topology-aware preferred allocation over real gRPC unix sockets with a fake kubelet."""

import os
import shutil
import tempfile
import threading
import time
from concurrent import futures

import grpc
import pytest

from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.operands import device_plugin as DPM
from gpu_operator_amd.operands import kubeletapi as K


@pytest.fixture
def short_tmp():
    d = tempfile.mkdtemp(prefix="dp-", dir="/tmp")   # unix socket paths must stay < 108 chars
    yield d
    shutil.rmtree(d, ignore_errors=True)


def cfg(**kw):
    return DPM.Config(**kw)


def test_discover_spx_uuid_ids(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r"))
    devs = DPM.discover(cfg(), root)
    assert len(devs) == 8 and {d.resource for d in devs} == {"amd.com/gpu"}
    assert devs[0].id.startswith("amdgpu-") and devs[0].render_minor == 128


def test_discover_cpx_single_and_mixed(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", compute="CPX"))
    assert {d.resource for d in DPM.discover(cfg(partition_strategy="single"), root)} == {"amd.com/gpu"}
    mixed = DPM.discover(cfg(partition_strategy="mixed"), root)
    assert len(mixed) == 64 and {d.resource for d in mixed} == {"amd.com/partition-cpx"}


def test_single_strategy_rejects_heterogeneous_partitions(tmp_path):
    root = fakesys.make_node(tmp_path / "r", n_gpus=2)
    # put GPU 1 in DPX
    from gpu_operator_amd import devices as D
    bdf = D.enumerate_gpus(str(root))[1]["pci_bdf"]
    D.set_partition(bdf, "compute", "DPX", root=str(root))
    with pytest.raises(ValueError, match="uniformly"):
        DPM.discover(cfg(partition_strategy="single"), str(root))
    assert {d.resource for d in DPM.discover(cfg(partition_strategy="mixed"), str(root))} == \
        {"amd.com/gpu", "amd.com/partition-dpx"}


def test_time_slicing_replicas(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=2))
    conf = tmp_path / "config.yaml"
    conf.write_text("version: v1\nsharing:\n  timeSlicing:\n    resources:\n    - name: amd.com/gpu\n      replicas: 4\n")
    c = DPM.Config.load(str(conf), {})
    devs = DPM.discover(c, root)
    assert len(devs) == 8 and devs[1].replica_of == devs[0].replica_of


def test_preferred_allocation_packs_partitions_of_one_gpu(tmp_path):
    root = str(fakesys.make_node(tmp_path / "r", compute="CPX"))
    devs = DPM.discover(cfg(partition_strategy="mixed"), root)
    # interleave GPUs in the available list; preference must still pick one physical GPU
    avail = sorted(devs, key=lambda d: (d.render_minor % 8, d.render_minor))
    ids = DPM.prefer(avail, [devs[9]], 8)
    chosen = [d for d in devs if d.id in ids]
    assert len({d.bdf for d in chosen}) == 1 and devs[9].id in ids


class FakeKubelet:
    def __init__(self, plugin_dir):
        self.registered = []
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self.server.add_generic_rpc_handlers((K.registration_handler(self.registered.append),))
        self.server.add_insecure_port("unix://" + os.path.join(plugin_dir, "kubelet.sock"))
        self.server.start()

    def stop(self):
        self.server.stop(0)


def test_grpc_register_list_allocate(tmp_path, short_tmp):
    root = str(fakesys.make_node(tmp_path / "r"))
    kubelet = FakeKubelet(short_tmp)
    p = DPM.DevicePlugin(cfg(), root=root, plugin_dir=short_tmp)
    try:
        p.start()
        assert [r.resource_name for r in kubelet.registered] == ["amd.com/gpu"]
        reg = kubelet.registered[0]
        assert reg.version == "v1beta1" and reg.options.get_preferred_allocation_available
        with grpc.insecure_channel("unix://" + os.path.join(short_tmp, reg.endpoint)) as ch:
            stub = K.device_plugin_stub(ch)
            stream = stub["ListAndWatch"](K.DP["Empty"]())
            first = next(stream)
            assert len(first.devices) == 8 and all(d.health == "Healthy" for d in first.devices)
            assert first.devices[0].topology.nodes[0].ID == 0
            ids = [first.devices[0].ID, first.devices[5].ID]
            req = K.DP["AllocateRequest"]()
            req.container_requests.add(devicesIDs=ids)
            resp = stub["Allocate"](req).container_responses[0]
            paths = sorted(d.container_path for d in resp.devices)
            assert paths == ["/dev/dri/renderD128", "/dev/dri/renderD133", "/dev/kfd"]
            assert resp.envs["AMD_VISIBLE_DEVICES"] == ",".join(sorted(ids))
            pref = K.DP["PreferredAllocationRequest"]()
            pref.container_requests.add(available_deviceIDs=[d.ID for d in first.devices], allocation_size=4)
            got = stub["GetPreferredAllocation"](pref).container_responses[0].deviceIDs
            assert len(got) == 4
            # health change (driver unloaded) is streamed
            os.remove(os.path.join(root, "sys/module/amdgpu/initstate"))
            p.check_health()
            upd = next(stream)
            assert all(d.health == "Unhealthy" for d in upd.devices)
            stream.cancel()
            bad = K.DP["AllocateRequest"]()
            bad.container_requests.add(devicesIDs=["nope"])
            with pytest.raises(grpc.RpcError):
                stub["Allocate"](bad)
    finally:
        p.stop()
        kubelet.stop()


def test_cdi_device_list_strategy(tmp_path, short_tmp):
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=1))
    p = DPM.DevicePlugin(cfg(device_list_strategy="cdi-cri"), root=root, plugin_dir=short_tmp)
    p.devices = DPM.discover(p.cfg, root)
    srv = DPM.ResourceServer("amd.com/gpu", p)
    req = K.DP["AllocateRequest"]()
    req.container_requests.add(devicesIDs=[p.devices[0].id])
    r = srv.Allocate(req, None).container_responses[0]
    assert [c.name for c in r.cdi_devices] == [f"amd.com/gpu={p.devices[0].id}"] and not r.devices
