"""srtp_mi355x_session_broadcast's two-rank control flow
(libsrtp_amd/csrc/srtp_host.c; SURVEY §8(e): session keys replicated to
every GPU) through the real C entry point, with two processes on the one
GPU of the box and tests/c/rccl_shim.so standing in for RCCL (which refuses
two ranks on one device): the length broadcast, the allocation agreement
(a max-reduction), the blob broadcast and the import.  The 8-GPU RCCL run
stays the driver's.  Each case runs under a time limit: no rank may hang."""
import json
import os
import subprocess
import sys
import tempfile

import pytest

from oracle import pyoracle as O
from tests.bcast_rank import batch, policies
from tests.test_gpu_parity import _gpu

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _two_ranks(case):
    d = tempfile.mkdtemp(prefix="srtp_bc_", dir="/tmp")
    sock = os.path.join(d, "s")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests",
                                                            "bcast_rank.py"),
                               str(r), sock, case,
                               os.path.join(d, "r%d.json" % r)], env=env,
                              cwd=ROOT)
             for r in range(2)]
    try:
        for p in procs:
            assert p.wait(timeout=120) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return [json.load(open(os.path.join(d, "r%d.json" % r))) for r in range(2)]


def test_broadcast_replica_equals_source():
    """rank 0's session (three AES-ICM streams, one AES-GCM stream, a
    template; advanced by a batch) reaches rank 1: both protect the next
    batch (incl. two new SSRCs the template clones) with identical bytes,
    equal to the oracle's; the replica re-exports the same blob"""
    _gpu()
    r0, r1 = _two_ranks("replica")
    assert r0["bcast"] == r1["bcast"] == "ok"
    assert r0["status"] == r1["status"] and r0["out"] == r1["out"]
    assert r0["blob"] == r1["blob"]
    assert r0["roc"] == r1["roc"]
    orc = O.Session(policies())
    for p in batch(1, 0xfff0):
        assert orc.protect(p, len(p) + 64)[0] == 0
    for i, p in enumerate(batch(2, 0x0020)):
        rc, ref = orc.protect(p, len(p) + 144)
        assert r0["status"][i] == rc
        assert rc or bytes.fromhex(r0["out"][i]) == ref, i


def test_broadcast_root_export_failure_all_ranks_fail():
    """the root has no session to export: it broadcasts length 0, so the
    other rank returns srtp_err_status_fail instead of waiting; the root
    returns bad_param"""
    _gpu()
    r0, r1 = _two_ranks("root_fail")
    assert "bad_param" in r0["bcast"], r0
    assert "fail" in r1["bcast"] and r1["bcast"] != "ok", r1


def test_broadcast_allocation_failure_all_ranks_fail():
    """rank 1 cannot allocate its blob buffers: the max-reduction of the
    failure flags makes BOTH ranks return srtp_err_status_alloc_fail before
    the blob broadcast (no rank left inside a collective)"""
    _gpu()
    r0, r1 = _two_ranks("alloc_fail")
    assert "alloc_fail" in r0["bcast"], r0
    assert "alloc_fail" in r1["bcast"], r1
