"""The multi-process launch of bench.py on the GPU box: real engine processes
(one context each, all on cuda:0 of the one-GPU box) over dist.py's TCP
control plane, message shards.  The 2-, 3- and 4-rank jobs'
whole-job record (counters, digest, coverage, forwards: gp_shard_combine)
must equal the 1-rank run's, and no process may load PyTorch."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--log2n", "16", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, extra=()):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GP_CTRL_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(world),
                                       *ARGS, *extra], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=180)
        assert p.returncode == 0, e[-3000:]
        outs.append(o)
    lines = [json.loads(x) for x in outs[0].splitlines() if x.startswith("{")]
    assert len(lines) == 1 and all(not o.strip() for o in outs[1:])
    return lines[0]


@pytest.mark.parametrize("world", [2, 3, 4])   # (the N = 8 launch is the driver's alone)
def test_multi_process_message_shards(world):
    """world ranks as the driver launches them at N = world (here all on the
    box's one GPU): the whole-job counters equal the one-process run's.  3
    ranks cut the 64 words 21 / 21 / 22 (rows of 32 words, partly used)."""
    one = _launch(1)
    many = _launch(world)
    assert many["n_gpus"] == world and f"message-shard x{world}" in many["config"]["parallelism"]
    for k in ("n", "arcs", "messages", "edge_deliveries_per_step", "rounds_per_step"):
        assert many["config"][k] == one["config"][k], k
    # the job's record, combined inside every step (gp_shard_combine over the
    # host all-gather: the ranks share the box's one GPU), equals the 1-GPU
    # run's: per-round receivers / senders as unions over the shards, the
    # per-vertex digest, per-message coverage and forwards (Peer.py:175-216)
    assert many["config"]["comm"]["comm_ranks"] == world
    assert many["config"]["comm"]["transport"].startswith("host")
    assert many["config"]["job"] == one["config"]["job"]
    w0 = 64 // world   # rank 0's words, rounded up to a power of two
    assert many["config"]["words_per_row"] == 1 << (w0 - 1).bit_length() and one["config"]["words_per_row"] == 64


def test_bench_process_loads_no_torch():
    code = ("import runpy, sys; sys.argv = ['bench.py'] + %r; "
            "runpy.run_path('bench.py', run_name='__main__'); "
            "sys.stderr.write('TORCH=%%s\\n' %% ('torch' in sys.modules))" % (ARGS,))
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "TORCH=False" in p.stderr
