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


def _health_stream(tmp_path, short_tmp, policy=None, n_gpus=8):
    root = str(fakesys.make_node(tmp_path / "r", n_gpus=n_gpus))
    kubelet = FakeKubelet(short_tmp)
    status = str(tmp_path / "validations")
    p = DPM.DevicePlugin(cfg(), root=root, plugin_dir=short_tmp, health_period=0.2, policy=policy, status_dir=status)
    p.start()
    return root, kubelet, p, status


def test_uncorrectable_ecc_withdraws_only_that_gpu_within_one_period(tmp_path, short_tmp):
    """ecc_uncorrectable goes up on GPU 3 -> ListAndWatch streams GPU 3 Unhealthy
    within one health period while the other seven stay Healthy; the reason reaches the status dir."""
    import json
    root, kubelet, p, status = _health_stream(tmp_path, short_tmp)
    t = threading.Thread(target=p.run_forever, daemon=True)
    t.start()
    try:
        reg = kubelet.registered[0]
        with grpc.insecure_channel("unix://" + os.path.join(short_tmp, reg.endpoint)) as ch:
            stream = K.device_plugin_stub(ch)["ListAndWatch"](K.DP["Empty"]())
            first = next(stream)
            assert all(d.health == "Healthy" for d in first.devices)
            gpu3 = p.devices[3].id
            fakesys.set_ras(root, 3, "umc", ue=1, ce=7)
            t0 = time.monotonic()
            upd = next(stream)
            took = time.monotonic() - t0
            health = {d.ID: d.health for d in upd.devices}
            assert health[gpu3] == "Unhealthy" and took < 0.2 + 0.5, took
            assert [i for i, h in health.items() if h != "Healthy"] == [gpu3]
            stream.cancel()
        with open(os.path.join(status, DPM.DEVICE_HEALTH_FILE)) as f:
            doc = json.load(f)
        assert doc["devices"][gpu3] == {"healthy": False, "reason": "uncorrectable RAS errors: 1 (umc)",
                                        "resource": "amd.com/gpu", "bdf": p.devices[3].bdf}
        assert sum(1 for d in doc["devices"].values() if d["healthy"]) == 7
    finally:
        p.stop()
        t.join(2)
        kubelet.stop()


def test_ras_in_any_block_and_retired_pages_withdraw_a_gpu(tmp_path, short_tmp):
    root, kubelet, p, status = _health_stream(tmp_path, short_tmp, policy=DPM.HealthPolicy(ue_max=0,
                                                                                          retired_pages_max=4))
    try:
        fakesys.set_ras(root, 1, "gfx", ue=2)                  # a compute-block uncorrectable error
        fakesys.add_bad_pages(root, 5, 3)                      # below the limit: still healthy
        fakesys.add_bad_pages(root, 6, 2, flag="P")            # pending pages do not count
        assert p.check_health()
        bad = {d.id: d.reason for d in p.devices if not d.healthy}
        assert bad == {p.devices[1].id: "uncorrectable RAS errors: 2 (gfx)"}
        fakesys.add_bad_pages(root, 5, 1)                      # the 4th retired page
        assert p.check_health()
        assert not p.devices[5].healthy and p.devices[5].reason == "retired HBM pages: 4 (limit 4)"
        assert not p.check_health()                            # no change, no stream update
        # the counts clear (driver reload): the device comes back
        fakesys.set_ras(root, 1, "gfx", ue=0)
        assert p.check_health() and p.devices[1].healthy and p.devices[1].reason == ""
    finally:
        p.stop()
        kubelet.stop()


def test_health_policy_from_env_and_a_sick_gpu_is_never_advertised(tmp_path, short_tmp):
    pol = DPM.HealthPolicy.from_env({"DP_HEALTH_UE_MAX": "5", "DP_HEALTH_RETIRED_PAGES_MAX": "-1"})
    assert (pol.ue_max, pol.retired_pages_max) == (5, -1)
    assert pol.verdict({"ras_ue_total": 5, "bad_pages_retired": 10 ** 6}) == ""
    assert pol.verdict({"ras_ue_total": 6, "ras_ue_blocks": "umc,xgmi_wafl"}).endswith("(umc,xgmi_wafl)")
    assert DPM.HealthPolicy(ue_max=-1).verdict({"ras_ue_total": 99}) == ""
    # already sick at start: the first ListAndWatch response carries Unhealthy
    root = str(fakesys.make_node(tmp_path / "r2", n_gpus=2))
    fakesys.set_ras(root, 0, "umc", ue=3)
    kubelet = FakeKubelet(short_tmp)
    p = DPM.DevicePlugin(cfg(), root=root, plugin_dir=short_tmp)
    try:
        p.start()
        assert [d.healthy for d in p.devices] == [False, True]
    finally:
        p.stop()
        kubelet.stop()
