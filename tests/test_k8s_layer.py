"""Fake API server semantics, selectors, merge patches, owner GC, watches, fault injection."""

import threading

import pytest

from gpu_operator_amd.k8s import errors
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.client import merge_patch
from gpu_operator_amd.k8s.fake import FakeClient


def cm(name, ns="ns", **labels):
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": ns, "labels": labels},
            "data": {"a": "1"}}


@pytest.mark.parametrize("sel,labels,ok", [
    ("app=x", {"app": "x"}, True),
    ("app==x", {"app": "y"}, False),
    ("app!=x", {}, True),
    ("app in (x, y),tier", {"app": "y", "tier": "a"}, True),
    ("app notin (x)", {"app": "x"}, False),
    ("!gpu", {"gpu": "1"}, False),
    ("!gpu,app=x", {"app": "x"}, True),
    ("amd.com/gpu.present=true", {"amd.com/gpu.present": "true"}, True),
    ({"matchLabels": {"a": "1"}, "matchExpressions": [{"key": "b", "operator": "Exists"}]}, {"a": "1", "b": ""}, True),
    ({"matchExpressions": [{"key": "b", "operator": "NotIn", "values": ["x"]}]}, {"b": "x"}, False),
    ({"a": "1"}, {"a": "1", "b": "2"}, True),
])
def test_label_selectors(sel, labels, ok):
    assert o.selector_matches(sel, labels) is ok


def test_invalid_selector():
    with pytest.raises(ValueError):
        o.parse_label_selector("a=b,,(")


def test_merge_patch_rfc7386():
    assert merge_patch({"a": 1, "b": {"c": 2, "d": 3}}, {"b": {"c": None, "e": 4}, "f": [1]}) == \
        {"a": 1, "b": {"d": 3, "e": 4}, "f": [1]}


def test_crud_resource_version_and_conflict():
    c = FakeClient()
    a = c.create(cm("x"))
    assert a["metadata"]["uid"] and a["metadata"]["resourceVersion"]
    with pytest.raises(errors.AlreadyExists):
        c.create(cm("x"))
    b = c.get("v1", "ConfigMap", "x", "ns")
    b["data"]["a"] = "2"
    c.update(b)
    a["data"]["a"] = "3"
    with pytest.raises(errors.Conflict):
        c.update(a)                     # stale resourceVersion
    assert c.get("v1", "ConfigMap", "x", "ns")["data"]["a"] == "2"
    c.delete("v1", "ConfigMap", "x", "ns")
    with pytest.raises(errors.NotFound):
        c.get("v1", "ConfigMap", "x", "ns")


def test_status_subresource_and_generation():
    c = FakeClient()
    ds = c.create({"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "d", "namespace": "ns"},
                   "spec": {"x": 1}})
    ds["status"] = {"numberUnavailable": 3}
    ds["spec"]["x"] = 2
    upd = c.update(ds)
    assert "status" not in upd and upd["metadata"]["generation"] == 2   # update ignores status
    upd["status"] = {"numberUnavailable": 0}
    st = c.update_status(upd)
    assert st["status"] == {"numberUnavailable": 0} and st["metadata"]["generation"] == 2


def test_owner_reference_garbage_collection_cascades():
    c = FakeClient()
    owner = c.create({"apiVersion": "amd.com/v1", "kind": "ClusterPolicy", "metadata": {"name": "cp"}})
    ds = {"apiVersion": "apps/v1", "kind": "DaemonSet", "metadata": {"name": "d", "namespace": "ns"}}
    o.set_controller_reference(owner, ds)
    ds = c.create(ds)
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "ns"}}
    o.set_controller_reference(ds, pod)
    c.create(pod)
    c.delete("amd.com/v1", "ClusterPolicy", "cp")
    assert c.objects("DaemonSet") == [] and c.objects("Pod") == []


def test_second_controller_reference_rejected():
    a = {"apiVersion": "v1", "kind": "X", "metadata": {"name": "a", "uid": "1"}}
    b = {"apiVersion": "v1", "kind": "X", "metadata": {"name": "b", "uid": "2"}}
    obj = {"metadata": {}}
    o.set_controller_reference(a, obj)
    o.set_controller_reference(a, obj)            # idempotent
    assert len(obj["metadata"]["ownerReferences"]) == 1
    with pytest.raises(ValueError):
        o.set_controller_reference(b, obj)


def test_list_filters_and_field_selectors():
    c = FakeClient([cm("a", app="x"), cm("b", app="y"), cm("c", ns="other", app="x")])
    assert [o.name(x) for x in c.list("v1", "ConfigMap", label_selector="app=x")] == ["a", "c"]
    assert [o.name(x) for x in c.list("v1", "ConfigMap", "ns", label_selector={"app": "x"})] == ["a"]
    assert [o.name(x) for x in c.list("v1", "ConfigMap", field_selector="metadata.name=b")] == ["b"]


def test_watch_delivers_initial_list_and_events():
    c = FakeClient([cm("a")])
    seen = []
    stop = c.watch("v1", "ConfigMap", lambda ev: seen.append((ev.type, o.name(ev.obj))))
    c.create(cm("b"))
    x = c.get("v1", "ConfigMap", "b", "ns")
    x["data"] = {}
    c.update(x)
    c.delete("v1", "ConfigMap", "a", "ns")
    stop()
    c.create(cm("z"))
    assert seen == [("ADDED", "a"), ("ADDED", "b"), ("MODIFIED", "b"), ("DELETED", "a")]


def test_fault_injection_interceptor():
    c = FakeClient([cm("a")])
    c.fail_on("get", "ConfigMap", errors.ApiError("boom", status=500), times=2)
    for _ in range(2):
        with pytest.raises(errors.ApiError):
            c.get("v1", "ConfigMap", "a", "ns")
    assert c.get("v1", "ConfigMap", "a", "ns")


def test_unserved_kind_raises_no_kind_match():
    c = FakeClient(unserved_kinds={"ServiceMonitor"})
    assert not c.has_kind("monitoring.coreos.com/v1", "ServiceMonitor")
    with pytest.raises(errors.NoKindMatch):
        c.list("monitoring.coreos.com/v1", "ServiceMonitor")


def test_patch_and_concurrent_updates_are_serialised():
    c = FakeClient([{"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n", "labels": {}}}])

    def worker(i):
        for j in range(20):
            c.patch("v1", "Node", "n", {"metadata": {"labels": {f"k{i}-{j}": "v"}}})
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert len(c.get("v1", "Node", "n")["metadata"]["labels"]) == 80


def test_stable_hash_ignores_key_order():
    assert o.stable_hash({"a": 1, "b": [1, 2]}) == o.stable_hash({"b": [1, 2], "a": 1})
    assert o.stable_hash({"a": 1}) != o.stable_hash({"a": 2})
