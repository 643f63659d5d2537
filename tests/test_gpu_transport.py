"""The RCCL transport's pieces on one MI355X.

* The exchange region's IPC mapping across PROCESSES: tools/ipc_check (built by
  __graft_entry__.build) allocates the region as engine.hip does (uncached device memory), exports
  its handle, and a second process opens it, checks the first one's words with system-scope loads
  and writes its own, which the first then checks — what a peer rank's k_pull_rows / k_recv_* rely
  on, minus the second GPU.
* The rest of the transport (count all-to-alls, the handle all-gather, the pulls, the quiet windows'
  allreduces) runs in the one-rank RCCL engine tests (test_gpu_parity.py / test_gpu_bench_parity.py
  `rccl`)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exchange_region_ipc_across_processes():
    exe = os.path.join(REPO, "tools", "ipc_check")
    if not os.path.exists(exe):
        pytest.skip("tools/ipc_check not built (__graft_entry__.build)")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC, as RCCL needs on this host
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    print(p.stdout.strip())
    assert p.returncode == 0 and "ipc_check ok" in p.stdout, p.stdout + p.stderr
    assert "uncached" in p.stdout, "the exchange region could not be allocated uncached"
