"""bench.py --gpus N: the launch decision and the rank launch command (CPU).

VERDICT r03 missing #1: ``--gpus`` used to be parsed and ignored, so a driver
run of ``bench.py --gpus 8`` timed one GPU.  Now the parent starts N ranks
itself (torch.distributed.run, one process per GPU) unless a launcher already
set WORLD_SIZE, and a launcher world that differs from --gpus is an error.
"""
import os
import subprocess
import sys

import pytest

import bench


def test_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, 1, "nccl") == ("rank", 1)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, 8, "nccl") == ("rank", 1)


def test_gpus_n_without_launcher_spawns_n_ranks():
    assert bench.launch_plan(8, {}, 8, "nccl") == ("spawn", 8)
    assert bench.launch_plan(2, {}, 1, "gloo") == ("spawn", 2)  # the one-GPU rehearsal


def test_inside_launcher_runs_as_rank():
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, 8, "nccl") == ("rank", 4)


@pytest.mark.parametrize("gpus,env,visible,backend", [
    (8, {"WORLD_SIZE": "1"}, 8, "nccl"),    # launcher world != --gpus
    (1, {"WORLD_SIZE": "2"}, 8, "nccl"),
    (8, {}, 1, "nccl"),                     # RCCL needs one GPU per rank
    (2, {"WORLD_SIZE": "2"}, 1, "nccl"),
    (0, {}, 1, "nccl"),
])
def test_mismatches_are_errors(gpus, env, visible, backend):
    with pytest.raises(SystemExit):
        bench.launch_plan(gpus, env, visible, backend)


def test_spawn_command_is_the_driver_form():
    cmd = bench.spawn_command(8, 29500, ["--gpus", "8", "--steps", "3"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29500" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3"]


def test_mismatch_exits_nonzero_before_any_gpu_work(tmp_path):
    """The real entry point: WORLD_SIZE=2 with --gpus 4 exits non-zero and
    prints no JSON line."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "4"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr and not p.stdout.strip()


def _n1_line():
    """The newest committed N = 1 default line with the cfg3_full sub-record."""
    import glob
    import json

    for path in sorted(glob.glob(os.path.join(os.path.dirname(bench.__file__), "profiles", "r0*", "**", "*.json"),
                                 recursive=True), reverse=True):
        try:
            with open(path) as f:
                rec = json.loads(f.readline())
        except (ValueError, OSError):
            continue
        if isinstance(rec, dict) and rec.get("n_gpus") == 1 and "cfg3_full" in (rec.get("sub") or {}):
            return rec
    return {"ms_per_step": 21.0, "sub": {"cfg3_full": {"ms_per_job": 170.0}}}  # round 4's measured line


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_scale_plan_fits_hbm_and_the_driver_limit(world):
    """the driver's first N = 8 run must fit one
    MI355X's 288 GB per rank and its 600 s, by the N = 1 measurements."""
    plan = bench.scale_plan(world, _n1_line())
    assert plan["fits_hbm"], plan
    assert plan["seconds"] < 600, plan
    if world == 8:  # the all-gather of a step (3.5 GB received per rank) stays below the reduction
        assert plan["allgather_ms_per_step"] < 2 * plan["step_ms"], plan


def test_init_process_group_has_a_timeout():
    """A stuck RCCL collective ends the rank (the process group watchdog)
    instead of hanging the driver's run: bench.py passes timeout=."""
    src = open(bench.__file__).read()
    assert 'init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)' in src
    assert "init_process_group(backend, timeout=tmo)" in src


def test_pipeline_summary_fields():
    """a rank's pipeline record -- overlap fraction
    (sum kernel + sum gather - wall) / sum gather and the all-gather's
    algorithm / bus bandwidth per plane -- from per-plane event times."""
    # two planes of 1M fp32 at N = 2: each all-gather writes 8 MB
    nbytes = [4 * 1_000_000 * 2] * 2
    hidden = bench.pipeline_summary(1, [10.0, 10.0], [2.0, 2.0], 22.0, nbytes, 2)
    assert hidden["rank"] == 1 and hidden["kernel_ms"] == 20.0 and hidden["allgather_ms"] == 4.0
    assert hidden["overlap_frac"] == 0.5  # (20 + 4 - 22) / 4: the first gather hid, the last did not
    assert hidden["allgather_algbw_gbs"] == 4.0 and hidden["allgather_busbw_gbs"] == 2.0
    inline = bench.pipeline_summary(0, [10.0, 10.0], [2.0, 2.0], 24.0, nbytes, 2)
    assert inline["overlap_frac"] == 0.0
    assert bench.pipeline_summary(0, [1.0], [], 1.0, [], 1)["overlap_frac"] is None  # one rank: no gather
    assert "reduction bound" in bench.gather_verdict([dict(hidden, overlap_frac=0.9)])
    assert "serialised" in bench.gather_verdict([inline])
    slow = bench.pipeline_summary(0, [10.0, 10.0], [15.0, 15.0], 40.0, nbytes, 2)
    assert "all-gather bound" in bench.gather_verdict([hidden, slow])


def test_gather_switch_parses():
    import sys as _sys

    saved = _sys.argv
    try:
        _sys.argv = ["bench.py", "--gpus", "2", "--gather", "inline"]
        assert bench.parse().gather == "inline"
        _sys.argv = ["bench.py", "--gpus", "2", "--gather", "p2p"]
        assert bench.parse().gather == "p2p"
        _sys.argv = ["bench.py"]
        assert bench.parse().gather == "overlap"
        # every leg maps to a stream policy and one of sharded's exchanges
        from p2pdl_amd import sharded

        assert set(bench.GATHER_LEGS) == {"overlap", "inline", "p2p"}
        assert all(ex in sharded.EXCHANGES for _, ex in bench.GATHER_LEGS.values())
    finally:
        _sys.argv = saved


def test_stdout_to_stderr_moves_native_prints(capfd):
    """bench's stdout is one JSON line: what native code prints to fd 1
    while the process group connects (gloo, RCCL debug) lands on stderr."""
    import os as _os

    with bench.stdout_to_stderr():
        _os.write(1, b"[Gloo] Rank 0 is connected\n")
    _os.write(1, b"{}\n")
    out, err = capfd.readouterr()
    assert out == "{}\n" and "[Gloo] Rank 0 is connected" in err
