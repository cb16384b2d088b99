"""Static validation of the Kubernetes deployment (no cluster here): every manifest
parses, names/ports/env line up across objects and with the package defaults, and
the contract the dashboard relies on holds (exporter on the node IP, Prometheus pod
name matching PROMETHEUS_METRICS_PODNAME's regex, kube-state-metrics scraped)."""

import os
import re

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K8S = os.path.join(ROOT, "deploy", "k8s")


def _docs(name):
    with open(os.path.join(K8S, name)) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def _all():
    out = {}
    for fn in sorted(os.listdir(K8S)):
        if fn.endswith(".yaml") and fn != "kustomization.yaml":
            for d in _docs(fn):
                out[(d["kind"], d["metadata"]["name"])] = d
    return out


def test_kustomization_lists_every_manifest():
    k = _docs("kustomization.yaml")[0]
    files = sorted(f for f in os.listdir(K8S) if f.endswith(".yaml") and f != "kustomization.yaml")
    assert sorted(k["resources"]) == files


def test_objects_have_namespace_and_selectors_match():
    objs = _all()
    for (kind, name), d in objs.items():
        if kind not in ("Namespace", "ClusterRole", "ClusterRoleBinding"):
            assert d["metadata"].get("namespace") == "monitoring", (kind, name)
        if kind in ("Deployment", "DaemonSet"):
            sel = d["spec"]["selector"]["matchLabels"]
            labels = d["spec"]["template"]["metadata"]["labels"]
            assert all(labels.get(k) == v for k, v in sel.items()), name
    for (kind, name), d in objs.items():
        if kind == "Service":
            sel = d["spec"]["selector"]
            assert any(
                k2 in ("Deployment", "DaemonSet")
                and all(o["spec"]["template"]["metadata"]["labels"].get(a) == b for a, b in sel.items())
                for (k2, _), o in objs.items()
            ), name


def test_exporter_daemonset_contract():
    from rocmdash import config

    ds = _all()[("DaemonSet", "rocmdash-exporter")]
    spec = ds["spec"]["template"]["spec"]
    assert spec["hostNetwork"] is True  # instance = <node-ip>:<port> (app.py:171)
    c = spec["containers"][0]
    port = c["ports"][0]["containerPort"]
    assert port == config.EXPORTER_PORT == int(ds["spec"]["template"]["metadata"]["annotations"]["prometheus.io/port"])
    assert "rocmdash.serve" in c["args"] and f"--port={port}" in c["args"]
    # the rank count follows the node (rocmdash.launch: one rank per physical GPU of the
    # KFD topology), never a hardcoded 8
    assert c["command"] == ["python3", "-m", "rocmdash.launch"]
    assert not any("nproc" in a for a in c["args"]) and "8" not in c["args"]
    assert "--node-window" in c["args"]  # a flag rocmdash.serve accepts
    # supervised ranks (partial-node operation): no torchrun whole-group restarts
    assert not any(a.startswith("--max-restarts") or a == "--torchrun" for a in c["args"]), c["args"]
    from rocmdash.launch import _split_module

    opts, module, margs = _split_module(c["args"])
    assert module == "rocmdash.serve" and any(o.startswith("--master-port=") for o in opts)
    assert any(o.startswith("--restart-base-s") for o in opts) and any(o.startswith("--restart-max-s") for o in opts)
    assert "amd.com/gpu" not in str(c.get("resources", {}))  # never takes GPUs from workloads
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # start-up is gated by a startupProbe sized for the node's placement calibration
    # (tests/test_placement.py holds the calibration to half of it); liveness only after it
    sp = c["startupProbe"]
    assert sp["httpGet"]["path"] == "/healthz" and sp["httpGet"]["port"] == port
    assert sp["periodSeconds"] * sp["failureThreshold"] >= 120
    assert "initialDelaySeconds" not in c["livenessProbe"]
    assert float(env["ROCMDASH_RCCL_INIT_TIMEOUT"]) < sp["periodSeconds"] * sp["failureThreshold"]
    mounts = {m["mountPath"] for m in c["volumeMounts"]}
    assert {"/dev/kfd", "/dev/dri", "/sys"} <= mounts


def test_prometheus_config_scrapes_exporter_and_ksm():
    objs = _all()
    cm = objs[("ConfigMap", "prometheus-config")]
    prom = yaml.safe_load(cm["data"]["prometheus.yml"])
    jobs = {j["job_name"]: j for j in prom["scrape_configs"]}
    assert {"amd-gpu-exporter", "kube-state-metrics"} <= set(jobs)
    keep = [r for r in jobs["amd-gpu-exporter"]["relabel_configs"] if r.get("action") == "keep"]
    assert any(r["regex"] == "rocmdash-exporter" for r in keep)
    ksm_svc = objs[("Service", "kube-state-metrics")]
    target = jobs["kube-state-metrics"]["static_configs"][0]["targets"][0]
    assert target == f"kube-state-metrics.monitoring.svc:{ksm_svc['spec']['ports'][0]['port']}"


def test_dashboard_env_points_at_prometheus():
    objs = _all()
    dep = objs[("Deployment", "rocmdash-dashboard")]
    env = {e["name"]: e["value"] for e in dep["spec"]["template"]["spec"]["containers"][0]["env"]}
    # the deployed page is the multi-panel view (BASELINE.json config #5), not the
    # reference's five panels: tests/test_deployed_path.py renders it with this env
    assert env.get("ROCMDASH_EXTENDED") == "1"
    svc = objs[("Service", "prometheus")]
    assert env["PROMETHEUS_METRICS_ENDPOINT"] == f"http://prometheus.monitoring.svc:{svc['spec']['ports'][0]['port']}/api/v1/query"
    # the reference's discovery regex ".*<PODNAME>.*" must match the Prometheus pod name
    pod_prefix = objs[("Deployment", "prometheus-server")]["metadata"]["name"]
    assert re.fullmatch(f".*{env['PROMETHEUS_METRICS_PODNAME']}.*", pod_prefix + "-5d8f7c9b4-abcde")
    # and Prometheus runs on the GPU node (discovery returns the Prometheus pod's host_ip)
    ps = objs[("Deployment", "prometheus-server")]["spec"]["template"]["spec"]
    ds = objs[("DaemonSet", "rocmdash-exporter")]["spec"]["template"]["spec"]
    assert ps["nodeSelector"] == ds["nodeSelector"]


def test_dockerfile_builds_native_runtime():
    with open(os.path.join(ROOT, "deploy", "docker", "Dockerfile")) as f:
        text = f.read()
    assert "rocmdash._build" in text and "gfx950" in text


@pytest.mark.parametrize("fn", sorted(f for f in os.listdir(K8S) if f.endswith(".yaml")))
def test_yaml_parses(fn):
    assert _docs(fn)


def test_module_entry_point_dispatch():
    import subprocess
    import sys

    res = subprocess.run([sys.executable, "-m", "rocmdash", "--help"], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert res.returncode == 0 and "serve" in res.stdout and "record" in res.stdout
    res = subprocess.run([sys.executable, "-m", "rocmdash", "nope"], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert res.returncode == 2
    res = subprocess.run([sys.executable, "-m", "rocmdash", "mock-prometheus", "--help"], cwd=ROOT, capture_output=True,
                         text=True, timeout=60)
    assert res.returncode == 0 and "usage" in res.stdout.lower()


def test_doctor_reports_every_check_and_fails_without_a_gpu():
    """``python -m rocmdash doctor --json``: every check reported; on a machine without a
    GPU the essential ones (topology, sysfs, hip) fail and the exit code says so."""
    import json
    import subprocess
    import sys

    res = subprocess.run([sys.executable, "-m", "rocmdash", "doctor", "--json", "--no-counters"], cwd=ROOT,
                         capture_output=True, text=True, timeout=120)
    d = json.loads(res.stdout.strip().splitlines()[-1])
    names = [c["check"] for c in d["checks"]]
    assert names == ["native", "topology", "numa", "sysfs", "amdsmi", "hip", "rccl", "kfd-proc"], names
    st = {c["check"]: c["status"] for c in d["checks"]}
    assert st["native"] == "ok" and st["rccl"] == "ok"
    import torch

    if not torch.cuda.is_available():
        assert res.returncode == 1 and not d["ok"] and st["topology"] == "FAIL" and st["hip"] == "FAIL"


def _quantity_mib(q: str) -> float:
    units = {"Ki": 1 / 1024, "Mi": 1, "Gi": 1024, "Ti": 1024 * 1024}
    for u, f in units.items():
        if q.endswith(u):
            return float(q[: -len(u)]) * f
    return float(q) / 2**20


def test_exporter_memory_limit_holds_the_measured_node():
    """The DaemonSet's memory request / limit against the production service as measured
    with 8 ranks (profiles/r06/nodecpu/node8_daemon.json: every node
    process's PSS - 8 ranks, the counter process, the supervisor - at amd-smi 10 Hz /
    counters 100 Hz). The limit keeps 25 % headroom over the measured node, the request
    half of it; the 1-GPU measurement scaled to 8 ranks fits too."""
    import json

    with open(os.path.join(ROOT, "profiles", "r06", "nodecpu", "node8_daemon.json")) as f:
        r8 = json.load(f)
    pss = r8["process_pss_mib"]
    assert len([k for k in pss if k.startswith("rank:")]) == 8 and r8["error"] is None
    node = sum(pss.values())
    assert abs(node - r8["node_pss_mib"]) <= 0.01 * node + 1, (node, r8["node_pss_mib"])
    c = _all()[("DaemonSet", "rocmdash-exporter")]["spec"]["template"]["spec"]["containers"][0]
    res = c["resources"]
    assert _quantity_mib(res["limits"]["memory"]) >= 1.25 * node, (res, node)
    assert _quantity_mib(res["requests"]["memory"]) >= 0.5 * node, (res, node)
    with open(os.path.join(ROOT, "profiles", "r05", "nodecpu", "node1_daemon.json")) as f:
        p1 = json.load(f)["process_pss_mib"]
    assert _quantity_mib(res["limits"]["memory"]) >= 1.25 * (8 * p1["rank:0"] + p1["counterd"] + p1["supervisor"])
