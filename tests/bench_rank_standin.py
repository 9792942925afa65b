"""TEST INFRASTRUCTURE: one bench.py rank with the GPU engine replaced by the
whole-grid oracle stand-in of test_bench_dist.py.  tests/test_bench_spawn.py
starts it through bench.spawn_ranks exactly as `bench.py --gpus N` (without
torch.distributed.run) starts bench.py itself."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE]

import mpi_amd  # noqa: E402
from mpi_amd import golhip  # noqa: E402
from test_bench_dist import _FakeEngine  # noqa: E402

golhip.Engine = _FakeEngine
golhip.unique_id = lambda: bytes(range(128))
mpi_amd.golhip = golhip
import bench  # noqa: E402

if os.environ.get("GOL_STANDIN_HANG_RANK") == os.environ.get("RANK"):
    # a rank that never arrives (a stuck RCCL group, a peer that died after
    # ncclCommInitRank): the others then wait for it at the first rendezvous
    import time
    time.sleep(3600)
sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
