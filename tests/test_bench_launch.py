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
