"""bench.py's multi-rank invocation with the overlapped-exchange leg (`sasrec_overlap`, sharded.py overlap_negatives),
rehearsed on one GPU: `--gpus 2 --backend gloo` launches two ranks that share cuda:0 (the driver's 8-GPU run uses
RCCL, one rank per GPU).  The headline and the leg both run the row-sharded SASRec step; the one JSON line carries the
leg with its own value and `overlap_negatives: true`, and the headline keeps the plain exchange."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_two_rank_bench_reports_the_overlapped_leg(tmp_path):
    full = tmp_path / "full.json"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--legs",
           "sasrec_overlap", "--cpu-baseline", "0", "--steps", "2", "--warmup", "1", "--batch", "64", "--seq-len", "50",
           "--items", "100000", "--eval-steps", "0", "--full-json", str(full)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2+rowshard2"
    leg = line["workloads"]["sasrec_overlap"]
    assert leg["value"] > 0
    res = json.loads(full.read_text())
    assert res["workloads"]["sasrec_overlap"]["config"]["overlap_negatives"] is True
    assert res["config"]["overlap_negatives"] is False
