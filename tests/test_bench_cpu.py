"""bench.py's host logic on CPU: the multi-rank launcher (`--gpus 2` starts two ranks
itself, gloo collectives in --dry-run), labels, and the build-keyed PMC record."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launcher_starts_ranks_and_gathers():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--dry-run", "--envs", "8"], capture_output=True, text=True, timeout=240,
                       env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1                         # rank 0 prints one line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["global_batch"] == 16
    assert out["episode_env_ids"] == [0, 8, 9]     # rank order, each rank's global ids
    assert out["counters"] == {"episodes_started": 8 + 1 + 8 + 2, "episodes_completed": 3,
                               "num_steps": 2 * 8 * 7}


def test_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--dry-run"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_labels():
    assert bench.metric_name(64, 64, 65536) == json.load(
        open(os.path.join(REPO, "BASELINE.json")))["metric"]
    assert "25×25" in bench.metric_name(25, 25, 4096)
    assert bench.step_kernel_name(64, 64, "none", "auto") == "k_env_step_bits64<false, 0>"
    assert bench.step_kernel_name(64, 64, "packed", "auto") == "k_env_step_bits64<true, 0>"
    assert bench.step_kernel_name(25, 25, "none", "auto") == "k_env_step_seg4<0, true>"
    assert bench.step_kernel_name(25, 29, "none", "auto") == "k_env_step_seg4<0, false>"
    assert bench.step_kernel_name(25, 40, "none", "auto") == "k_env_step_small<0>"
    assert bench.step_kernel_name(128, 128, "none", "auto") == "k_env_step_bits128<0>"
    assert (bench.step_kernel_name(128, 128, "none", "auto", "stream")
            == "k_env_step_bits128<3>")                  # draws decided before the step
    assert (bench.step_kernel_name(64, 64, "none", "auto", "stream")
            == "k_env_step_bits64<false, 1>")
    # replay without any spawner runs the Philox form
    assert (bench.step_kernel_name(64, 64, "none", "auto", "stream", replay=False)
            == "k_env_step_bits64<false, 0>")
    assert bench.step_kernel_name(64, 64, "none", "generic") == "k_env_step_generic"


def test_pmc_record_keyed_on_build(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    rec = {"kernel": "void k_env_step_bits64<false, 0>(StepKArgs)", "build_id": "abc",
           "hbm_bytes_per_launch": 123.0, "profile": "rX"}
    (prof / "pmc_c3.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.traffic_from_record("c3", "none", "abc", "k_env_step_bits64<false, 0>")[0] == 123.0
    # replay lines keep their own record
    assert bench.traffic_from_record("c3", "none", "abc", "k_env_step_bits64<false, 0>",
                                     "stream")[0] is None
    assert bench.traffic_from_record("c3", "none", "other", "k_env_step_bits64<false, 0>")[0] is None
    assert bench.traffic_from_record("c3", "none", "abc", "k_env_step_bits128<0>")[0] is None
    assert bench.traffic_from_record("c5", "none", "abc", "k_env_step_bits128<0>")[0] is None


def test_build_id_file_matches_library():
    from safelife_amd import _lib
    _lib.build()
    bid = bench.file_build_id()
    assert bid and len(bid) == 16
    assert _lib.build_id() == bid
