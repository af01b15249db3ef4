"""bench.py's launch contract on CPU (no GPU call): --gpus N means N ranks."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_world_size_mismatch_fails_before_any_gpu_call():
    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "--gpus 2 but WORLD_SIZE=1" in r.stderr


def test_gpus_n_launches_n_ranks(monkeypatch):
    import bench
    seen = {}

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd

        class R:
            returncode = 0
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    a = type("A", (), {"gpus": 4})()
    assert bench.launch_ranks(a) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_stale_pmc_summary_is_not_reported(tmp_path, monkeypatch):
    import json
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "zz_pmc_cfg2.json").write_text(json.dumps({"source_sha256": "0" * 64,
                                                       "cfg2": {"gru_bwd": {"hbm_bytes_per_launch": 1e8}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "kernel_source_hash", lambda: "1" * 64)
    v, why = bench.pmc_traffic("cfg2", "gru_bwd")
    assert v is None and "stale" in why
    monkeypatch.setattr(bench, "kernel_source_hash", lambda: "0" * 64)
    v, why = bench.pmc_traffic("cfg2", "gru_bwd")
    assert v == 1e8 and "zz_pmc_cfg2.json" in why
