"""bench.py's multi-rank launch logic on the CPU (no GPU): `--gpus N` without a launcher starts N rank processes
itself, a launcher's WORLD_SIZE must agree with --gpus, a failing rank stops the others, and the stdout line stays
compact enough for the driver's tail."""
import importlib.util
import json
import os
import sys
import time
from types import SimpleNamespace

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_resolve_world(bench):
    a = SimpleNamespace(gpus=1)
    assert bench.resolve_world(a, {}) == (1, False)
    assert bench.resolve_world(SimpleNamespace(gpus=8), {}) == (8, True)
    assert bench.resolve_world(SimpleNamespace(gpus=2), {"WORLD_SIZE": "2"}) == (2, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(SimpleNamespace(gpus=1), {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.resolve_world(SimpleNamespace(gpus=8), {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.resolve_world(SimpleNamespace(gpus=0), {})


def test_rank_envs(bench):
    envs = bench.rank_envs(4, 29999, base={"HSA_ENABLE_IPC_MODE_LEGACY": "0", "WORLD_SIZE": "x"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999"
               and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)


CHILD = r'''
import os, sys, time
out = sys.argv[1]
r, w = os.environ["RANK"], os.environ["WORLD_SIZE"]
with open(os.path.join(out, f"rank{r}"), "w") as f:
    f.write(f"{r} {w} {os.environ['LOCAL_RANK']} {os.environ['MASTER_ADDR']}")
if len(sys.argv) > 2 and sys.argv[2] == "fail":
    if r == "1":
        sys.exit(3)
    time.sleep(60)
'''


def test_launch_ranks_runs_every_rank(bench, tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    args = SimpleNamespace(gpus=3, backend="gloo")
    rc = bench.launch_ranks(args, argv=[str(tmp_path)], script=str(script))
    assert rc == 0
    got = sorted((tmp_path / f"rank{r}").read_text() for r in range(3))
    assert got == ["0 3 0 127.0.0.1", "1 3 1 127.0.0.1", "2 3 2 127.0.0.1"]


def test_launch_ranks_stops_the_others_when_one_fails(bench, tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    t0 = time.time()
    rc = bench.launch_ranks(SimpleNamespace(gpus=2, backend="gloo"), argv=[str(tmp_path), "fail"], script=str(script))
    assert rc == 3
    assert time.time() - t0 < 30  # rank 0 (sleeping 60 s) was terminated, not waited for


def test_launch_ranks_refuses_more_gpus_than_visible(bench, tmp_path):
    import torch
    if torch.cuda.device_count() >= 64:
        pytest.skip("machine has many GPUs")
    assert bench.launch_ranks(SimpleNamespace(gpus=64, backend="nccl"), argv=[], script=str(tmp_path / "x.py")) == 2


def _fake_roof(name, frac, ms):
    return {"kernel": name, "bound": "hbm", "achieved": 1.0, "peak": 8000.0, "unit": "GB/s", "frac": frac,
            "traffic": 1, "avg_ms": ms, "launches": 2, "total_ms": 2 * ms, "bytes_per_launch": 1.0}


def test_compact_line_keeps_contract_and_every_workload(bench):
    roofs = [_fake_roof(f"k{i}", 0.5, 1.0 / (i + 1)) for i in range(25)]
    roofs.append(_fake_roof("asme_embedding_ln_fwd", 0.61, 0.01))
    leg = {"metric": "m", "value": 1.0, "unit": "sequences/s", "ms_per_step": 2.0, "n_gpus": 2,
           "config": {"parallelism": "dp2"}, "rooflines": roofs, "roofline": roofs[0],
           "cpu_baseline": {"value": 3.0, "cores": 16, "kind": "port", "batch": 64, "s_per_step": 1.0,
                            "sample": "x" * 500}}
    result = {"metric": "training sequences/sec", "value": 123.0, "unit": "sequences/s", "n_gpus": 2, "steps": 3,
              "warmup": 1, "ms_per_step": 1.0, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
              "dtype": "fp32", "data": "synthetic", "config": {"workload": "w", "parallelism": "dp2+rowshard2"},
              "roofline": roofs[0], "rooflines": roofs, "cpu_baseline": None,
              "eval": {"metric": "e", "value": 9.0, "unit": "sequences/s", "ms_per_step": 3.0, "steps": 3,
                       "ndcg@10": 0.0, "roofline": roofs[0], "rooflines": roofs},
              "workloads": {"bert4rec": leg, "kebert4rec": leg, "sasrec_zipf": leg, "sasrec_overlap": leg}}
    c = bench.compact(result)
    line = json.dumps(c)
    assert len(line) < 6000
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "config", "roofline", "cpu_baseline"):
        assert k in c
    assert set(c["workloads"]) == {"bert4rec", "kebert4rec", "sasrec_zipf", "sasrec_overlap"}
    assert all(len(w["rooflines_top"]) == 3 and w["value"] == 1.0 for w in c["workloads"].values())
    assert c["target_kernels"]["asme_embedding_ln_fwd"] == 0.61
    assert c["eval"]["value"] == 9.0


def test_default_legs_include_the_overlapped_exchange(bench):
    """the default invocation measures the overlapped row exchange beside the headline wherever rows cross the fabric
    (the leg is skipped at N = 1); an unknown leg name is refused"""
    legs = dict(bench.parse_legs(bench.build_parser().get_default("legs")))
    assert {"bert4rec", "kebert4rec", "sasrec_zipf", "sasrec_overlap"} <= set(legs)
    with pytest.raises(SystemExit):
        bench.parse_legs("sasrec_overlapped")
