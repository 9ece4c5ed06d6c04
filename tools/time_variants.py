#!/usr/bin/env python3
"""Times the protect kernels of several libsrtp_mi355x.so builds (exp_build/
<name>/) on the bench workload; prints kernel ms per 1M x 1400B batch.
Timing-only: variants may be deliberately incorrect (experiments)."""
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, os, json
sys.path.insert(0, %r)
import torch
assert os.environ["LIBSRTP_MI355X_LIB"] == %r
import libsrtp_amd.srtp as S
assert S.lib()._name == os.environ["LIBSRTP_MI355X_LIB"]
import bench
L = S
pol, payload, n, tag = bench.CONFIGS[%r]
n = %d
sess = S.Session([dict(pol, ssrc_type=1, ssrc=0xcafebabe, window_size=128,
                      allow_repeat_tx=0, keys=[bench.TEST_KEY])])
rtp_len = 12 + payload; slot = (rtp_len + tag + 15) & ~15
dev = torch.device("cuda", 0)
arena = torch.randint(0, 256, (n, slot), dtype=torch.uint8, device=dev)
arena[:, 0] = 0x80; arena[:, 1] = 96
arena[:, 8:12] = torch.tensor([0xca, 0xfe, 0xba, 0xbe], dtype=torch.uint8, device=dev)
off = torch.arange(n, dtype=torch.int64, device=dev) * slot
ln = torch.full((n,), rtp_len, dtype=torch.int32, device=dev)
ol = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
idx = torch.arange(n, dtype=torch.int64, device=dev)
sess.set_timing(True)
ks = []
for it in range(24):
    seq = (idx + 0x1234 + it * n) & 0xffff
    arena[:, 2] = (seq >> 8).to(torch.uint8); arena[:, 3] = (seq & 0xff).to(torch.uint8)
    ol.fill_(slot)
    flat = arena.view(-1)
    assert sess.protect_device(flat, off, ln, flat, off, ol, st) == 0
    ks.append(sess.last_kernel_ms())
tail = sorted(ks[8:])
print(json.dumps({"kernel_ms": tail[len(tail) // 2], "min": tail[0]}))
'''


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        # one build in this process (for rocprofv3 -- python3 ... --one NAME)
        name, cfg = sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "icm128"
        so = os.path.join(ROOT, "libsrtp_amd", "libsrtp_mi355x.so") \
            if name == "tree" else os.path.join(ROOT, "exp_build", name,
                                                "libsrtp_mi355x.so")
        os.environ["LIBSRTP_MI355X_LIB"] = so
        exec(CHILD % (ROOT, so, cfg, 1 << 20), {"__name__": "child"})
        return
    cfg = sys.argv[1] if len(sys.argv) > 1 else "icm128"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    names = sorted(os.listdir(os.path.join(ROOT, "exp_build"))) \
        if os.path.isdir(os.path.join(ROOT, "exp_build")) else []
    runs = [(nm, os.path.join(ROOT, "exp_build", nm, "libsrtp_mi355x.so"), {})
            for nm in names]
    # the in-tree build for reference
    runs.append(("tree", os.path.join(ROOT, "libsrtp_amd", "libsrtp_mi355x.so"), {}))
    for name, so, extra in runs:
        code = CHILD % (ROOT, so, cfg, n)
        env = dict(os.environ, LIBSRTP_MI355X_LIB=so, **extra)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True,
                           text=True, timeout=300, env=env)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-400:]
        print(name, cfg, line, flush=True)


if __name__ == "__main__":
    main()
