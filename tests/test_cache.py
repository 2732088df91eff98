"""Informer cache (runtime/cache.py): reconcile reads served from watch-fed stores.

Reference bar: main.go:104 (the controller-runtime manager's cached client). Done-criterion of
the round-1 review: on a 500-node cluster an unchanged steady-state pass makes no API reads
and at most a small constant number of writes.
"""

import time

import pytest

from gpu_operator_amd.controllers import consts as C
from gpu_operator_amd.k8s import errors
from gpu_operator_amd.k8s import objects as o
from gpu_operator_amd.k8s.fake import FakeClient
from gpu_operator_amd.k8s.sim import ClusterSim
from gpu_operator_amd.runtime.cache import CachedClient
from k8s_helpers import NS, cluster, gpu_node, reconciler


def _verbs(calls, verbs):
    return [c for c in calls if c[0] in verbs]


WRITES = ("create", "update", "update_status", "delete", "evict")


@pytest.mark.parametrize("n_nodes", [500])
def test_steady_state_pass_makes_no_api_reads(n_nodes):
    raw = cluster([gpu_node(f"node-{i:04d}") for i in range(n_nodes)])
    c = CachedClient(raw)
    rec = reconciler(c)
    sim = ClusterSim(raw)                 # the simulated kubelet/DS controller talk to the API directly
    for _ in range(6):
        rec.reconcile(("", "cluster-policy"))
        sim.sync()
        if raw.get("amd.com/v1", "ClusterPolicy", "cluster-policy").get("status", {}).get("state") == "ready":
            break
    assert raw.get("amd.com/v1", "ClusterPolicy", "cluster-policy")["status"]["state"] == "ready"
    rec.reconcile(("", "cluster-policy"))            # settle
    raw.calls.clear()
    c.reset_stats()
    t0 = time.perf_counter()
    rec.reconcile(("", "cluster-policy"))
    dt = time.perf_counter() - t0
    reads = _verbs(raw.calls, ("get", "list"))
    writes = _verbs(raw.calls, WRITES)
    assert reads == [] and c.stats() == {"get": 0, "list": 0}, reads[:10]
    assert len(writes) <= 2, writes                  # nothing changed: (almost) nothing written
    print(f"\n{n_nodes} nodes: steady-state pass {dt * 1e3:.0f} ms, {len(writes)} writes, 0 API reads")


def test_uncached_client_pays_reads_every_pass():
    """The same pass without the cache: the cost the informers remove."""
    raw = cluster([gpu_node(f"node-{i}") for i in range(20)])
    rec = reconciler(raw)
    sim = ClusterSim(raw)
    for _ in range(6):
        rec.reconcile(("", "cluster-policy"))
        sim.sync()
    raw.calls.clear()
    rec.reconcile(("", "cluster-policy"))
    assert len(_verbs(raw.calls, ("get", "list"))) > 50


def test_cache_reads_its_own_writes_and_tracks_watch_events():
    raw = FakeClient([gpu_node("a")])
    c = CachedClient(raw)
    assert [o.name(n) for n in c.list("v1", "Node")] == ["a"]
    c.patch("v1", "Node", "a", {"metadata": {"labels": {"x": "1"}}})
    assert o.get_labels(c.get("v1", "Node", "a"))["x"] == "1"
    raw.create(gpu_node("b"))                        # someone else's write arrives by watch
    assert [o.name(n) for n in c.list("v1", "Node", label_selector={"x": "1"})] == ["a"]
    assert {o.name(n) for n in c.list("v1", "Node")} == {"a", "b"}
    raw.delete("v1", "Node", "b")
    with pytest.raises(errors.NotFound):
        c.get("v1", "Node", "b")
    # returned objects are copies
    n = c.get("v1", "Node", "a")
    n["metadata"]["labels"]["x"] = "mutated"
    assert o.get_labels(c.get("v1", "Node", "a"))["x"] == "1"
    assert c.stats() == {"get": 0, "list": 1}        # the informer's single initial LIST


def test_cache_ignores_older_events_and_passes_through_unserved_kinds():
    raw = FakeClient([gpu_node("a")], unserved_kinds={"ClusterVersion"})
    c = CachedClient(raw)
    cur = c.get("v1", "Node", "a")
    inf = c._informers[("v1", "Node")]
    stale = dict(cur, metadata=dict(cur["metadata"], resourceVersion="0", labels={"stale": "yes"}))
    inf._upsert(stale)
    assert "stale" not in o.get_labels(c.get("v1", "Node", "a"))
    with pytest.raises(errors.NoKindMatch):
        c.get("config.openshift.io/v1", "ClusterVersion", "version")
    with pytest.raises(errors.NoKindMatch):
        c.get("config.openshift.io/v1", "ClusterVersion", "version")
    assert c.stats()["get"] == 2                     # passed through, not cached
    # Leases bypass the cache (leader election needs fresh reads)
    raw.create({"apiVersion": "coordination.k8s.io/v1", "kind": "Lease", "metadata": {"name": "l", "namespace": NS}})
    c.get("coordination.k8s.io/v1", "Lease", "l", NS)
    assert ("coordination.k8s.io/v1", "Lease") not in c.cached_kinds()


def test_controller_watch_shares_the_informer_stream():
    raw = FakeClient([gpu_node("a")])
    c = CachedClient(raw)
    seen = []
    stop = c.watch("v1", "Node", lambda ev: seen.append((ev.type, o.name(ev.obj))))
    raw.create(gpu_node("b"))
    stop()
    raw.create(gpu_node("c"))
    assert seen == [("ADDED", "a"), ("ADDED", "b")]
    assert sum(1 for w in raw._watchers if w[1] == "Node") == 1


def test_cached_client_over_http_api_server():
    """RestClient + informers against the in-process API server: events arrive asynchronously."""
    from gpu_operator_amd.k8s.apiserver import FakeAPIServer
    from gpu_operator_amd.k8s.rest import Config, RestClient
    srv = FakeAPIServer(FakeClient([gpu_node("a")]))
    srv.start()
    try:
        c = CachedClient(RestClient(Config(host=srv.url)))
        assert [o.name(n) for n in c.list("v1", "Node")] == ["a"]
        srv.client.create(gpu_node("b"))
        deadline = time.time() + 10
        while time.time() < deadline and len(c.list("v1", "Node")) < 2:
            time.sleep(0.05)
        assert {o.name(n) for n in c.list("v1", "Node")} == {"a", "b"}
        c.patch("v1", "Node", "a", {"metadata": {"labels": {"k": "v"}}})
        assert o.get_labels(c.get("v1", "Node", "a"))["k"] == "v"      # own write visible at once
        c.stop()
    finally:
        srv.stop()
