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
    # the 64x64 board in bit planes (round 6): the instance for the planes the pool keeps
    assert (bench.step_kernel_name(64, 64, "none", "auto", keep=0x877F)
            == "k_env_step_bits64_planes<34687u, 0>")
    assert (bench.step_kernel_name(64, 64, "none", "auto", keep=0x1234)
            == "k_env_step_bits64_planes<0u, 0>")
    assert (bench.step_kernel_name(64, 64, "none", "auto", planes=False)
            == "k_env_step_bits64<0, 0>")
    assert (bench.step_kernel_name(64, 64, "packed", "auto", keep=0x877F)
            == "k_env_step_bits64_planes<34687u, 1>")
    assert (bench.step_kernel_name(64, 64, "packed", "auto", planes=False)
            == "k_env_step_bits64<1, 0>")
    assert bench.step_kernel_name(25, 25, "none", "auto") == "k_env_step_seg4<0, true>"
    assert bench.step_kernel_name(25, 29, "none", "auto") == "k_env_step_seg4<0, false>"
    assert bench.step_kernel_name(25, 40, "none", "auto") == "k_env_step_small<0>"
    assert (bench.step_kernel_name(128, 128, "none", "auto", keep=0x07FB)
            == "k_env_step_bits128<0, 2043u>")         # the C5 planes' instance
    assert (bench.step_kernel_name(128, 128, "none", "auto", keep=0xFFFF)
            == "k_env_step_bits128<0, 65535u>")
    assert (bench.step_kernel_name(128, 128, "none", "auto", "stream", keep=0x07FB)
            == "k_env_step_bits128<3, 2043u>")         # draws decided before the step
    assert (bench.step_kernel_name(128, 128, "packed", "auto", keep=0x07FB)
            == "k_env_step_bits128_view<0, 2043u>")
    assert (bench.step_kernel_name(64, 64, "none", "auto", "stream")
            == "k_env_step_bits64<0, 1>")
    # replay without any spawner runs the Philox form (in planes)
    assert (bench.step_kernel_name(64, 64, "none", "auto", "stream", replay=False,
                                   keep=0xFFFF) == "k_env_step_bits64_planes<65535u, 0>")
    assert bench.step_kernel_name(64, 64, "none", "generic") == "k_env_step_generic"
    # channel views are written by the step kernel (obs_kind 2: u16 / bf16, 3: u8, 4: f32)
    assert bench.step_kernel_name(64, 64, "channels", "auto") == "k_env_step_bits64<2, 0>"
    assert (bench.step_kernel_name(64, 64, "channels", "auto", obs_dtype="bfloat16")
            == "k_env_step_bits64<2, 0>")
    assert (bench.step_kernel_name(64, 64, "channels", "auto", obs_dtype="uint8")
            == "k_env_step_bits64<3, 0>")


def test_pmc_record_keyed_on_build(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    rec = {"kernel": "void k_env_step_bits64<0, 0>(StepKArgs)", "build_id": "abc",
           "hbm_bytes_per_launch": 123.0, "profile": "rX"}
    (prof / "pmc_c3.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.traffic_from_record("c3", "none", "abc", "k_env_step_bits64<0, 0>")[0] == 123.0
    # replay lines keep their own record
    assert bench.traffic_from_record("c3", "none", "abc", "k_env_step_bits64<0, 0>",
                                     "stream")[0] is None
    assert bench.traffic_from_record("c3", "none", "other", "k_env_step_bits64<0, 0>")[0] is None
    assert bench.traffic_from_record("c3", "none", "abc", "k_env_step_bits128<0>")[0] is None
    assert bench.traffic_from_record("c5", "none", "abc", "k_env_step_bits128<0>")[0] is None


def test_build_id_file_matches_library():
    from safelife_amd import _lib
    _lib.build()
    bid = bench.file_build_id()
    assert bid and len(bid) == 16
    assert _lib.build_id() == bid


def test_cache_resident_configs_claim_no_hbm_fraction():
    """C2 (4 096 x 25x25, ~15 MB of state) stays in the Infinity Cache: bench.py prints
    roofline.bound "cache" with no frac and times its kernel over one bracket of all
    timed steps (so kernel_ms <= ms_per_step); the HBM configs keep "hbm"."""
    assert bench.roofline_bound(25, 25, 4096) == "cache"
    assert bench.roofline_bound(64, 64, 65536) == "hbm"
    assert bench.roofline_bound(64, 64, 32768) == "hbm"          # C4's shard
    assert bench.roofline_bound(128, 128, 65536) == "hbm"
    assert bench.state_bytes(25, 25, 4096) < bench.CACHE_RESIDENT_BYTES


def test_seeded_replay_names():
    """--rng seeded runs the replay kernels with the device generator; its PMC record
    is its own."""
    assert (bench.step_kernel_name(128, 128, "none", "auto", "seeded", keep=0x07FB)
            == "k_env_step_bits128<3, 2043u>")
    assert bench.pmc_record_path("c5", "none", "seeded").endswith("pmc_c5_seeded.json")
    assert bench.pmc_record_path("c5", "none", "stream").endswith("pmc_c5_stream.json")


def test_c1_cpu_leg_single_level():
    """C1's CPU chain leg takes the single 25x25 level file (one env, one thread)."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--cpu-leg", json.dumps(
        {"pools": [os.path.join(REPO, "tests", "golden", "levels", bench.C1_LEVEL)],
         "threads": 1, "envs": 1, "seconds": 0.3,
         "kw": {"time_limit": 1000, "view_shape": [33, 33], "penalty_coef": 1.0,
                "min_performance": 0.01}})], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["n"] > 0 and r["rate"] > 0
