"""The captured data-parallel step (graphs.StepGraph with SyncBatchNorm statistics and the
gradient all-reduce as RCCL collectives inside the graph, no DDP) on a one-rank group equals
the single-process step (tools/dp_graph_check.py, run in its own process because it
initialises a process group), and bench.py keeps exactly one JSON line on stdout with the
RCCL communicator up."""
import json
import os
import subprocess
import sys

import pytest

from helpers import ROOT

pytestmark = pytest.mark.gpu


def test_dp_graph_step_equals_single_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "dp_graph_check.py")],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "OK dp-graph" in r.stdout


def test_bench_dp_collectives_one_json_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dp-collectives",
                        "--steps", "3", "--warmup", "2", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["value"] > 0 and res["n_gpus"] == 1


def test_capture_after_eager_collectives_on_dedicated_streams():
    """Round 6: the watchdog abort's mechanism (tools/pg_capture_probe.py: an eager blocking
    collective's end event sits on the stream it was issued from; if that stream joins a capture
    before the watchdog retired the work, the watchdog's query aborts the process) and its fix
    (dist.dedicated_stream: eager and capture roles never share a stream).  The probe issues
    eager collectives and immediately captures the same collectives, holding the capture open
    across ~15 watchdog passes: with the product's streams it must not abort."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pg_capture_probe.py"),
                        "product"], capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "product: ok" in r.stdout
