#!/usr/bin/env python3
"""Probe: which consecutive srtp_protect_device batches stay on the device
pre-pass for round-robin multi-stream batches (streams x per-stream)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libsrtp_amd as L
import bench


def run(ns, per, batches=4, payload=160):
    pol, _, _, tag = bench.CONFIGS["g711"]
    base = 0x10000000
    sess = L.Session([dict(pol, ssrc_type=1, ssrc=base + k, window_size=128,
                           allow_repeat_tx=0, keys=[key])
                      for k, key in enumerate(bench.stream_keys(ns, 1))])
    n = ns * per
    rtp_len = 12 + payload
    slot = (rtp_len + tag + 15) & ~15
    dev = torch.device("cuda", 0)
    arena = torch.randint(0, 256, (n, slot), dtype=torch.uint8, device=dev)
    arena[:, 0] = 0x80
    arena[:, 1] = 96
    idx = torch.arange(n, dtype=torch.int64, device=dev)
    pk_ssrc = base + idx % ns
    for k in range(4):
        arena[:, 8 + k] = ((pk_ssrc >> (24 - 8 * k)) & 0xff).to(torch.uint8)
    pk_seq = idx // ns
    off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    ln = torch.full((n,), rtp_len, dtype=torch.int32, device=dev)
    ol = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    hist = []
    prev = (0, 0)
    for b in range(batches):
        seq = (pk_seq + 0x1234 + b * per) & 0xffff
        arena[:, 2] = (seq >> 8).to(torch.uint8)
        arena[:, 3] = (seq & 0xff).to(torch.uint8)
        ol.fill_(slot)
        flat = arena.view(-1)
        assert sess.protect_device(flat, off, ln, flat, off, ol, st) == 0
        d, h = sess.prepass_stats()
        path = "D" if d > prev[0] else "H"
        prev = (d, h)
        vals, cnt = torch.unique(st, return_counts=True)
        errs = {int(v): int(c) for v, c in zip(vals.cpu(), cnt.cpu()) if v != 0}
        hist.append("%s%s" % (path, errs or ""))
    print("streams %6d per %4d: %s" % (ns, per, " ".join(hist)), flush=True)


if __name__ == "__main__":
    cases = [(1, 1 << 21), (16384, 128), (65536, 128), (65536, 6)]
    if len(sys.argv) > 1:
        cases = [tuple(int(x) for x in a.split("x")) for a in sys.argv[1:]]
    for ns, per in cases:
        run(ns, per, batches=2)
    print("last abort", flush=True)
