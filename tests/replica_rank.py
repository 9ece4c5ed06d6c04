"""One rank of tests/test_gpu_replica.py::test_two_ranks_vs_oracle (run by
torch.distributed.run with SRTP_BENCH_DEVICE=0 and gloo, two ranks on one
GPU).  Rank 0 creates the AES-256-GCM session holding both ranks' streams;
bench.replicate_session carries it to rank 1 (srtp_mi355x_session_export /
_import); each rank keeps its own stream, protects 8192 packets of it on the
device and saves inputs and outputs for the parent's oracle check."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_dir):
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    import libsrtp_amd as L
    from tests.test_gpu_parity import policy

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("SRTP_BENCH_DEVICE", rank)))
    dist.init_process_group("gloo")
    dev = torch.device("cuda", torch.cuda.current_device())
    pols = [policy("gcm256_16", ssrc=bench.rank_ssrc(r), seed=11)
            for r in range(world)]
    sess, how = bench.replicate_session(L, pols, world, rank, dev, "gloo")
    for r in range(world):
        if r != rank:
            assert sess.remove_stream(bench.rank_ssrc(r)) == 0
    n, payload, tag = 8192, 1400, 16
    slot = (12 + payload + tag + 15) & ~15
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    a = torch.randint(0, 256, (n, slot), dtype=torch.uint8, device=dev,
                      generator=g)
    seq = (torch.arange(n, device=dev) + 0xff00 + 977 * rank) & 0xffff
    a[:, 0], a[:, 1] = 0x80, 96
    a[:, 2], a[:, 3] = (seq >> 8).to(torch.uint8), (seq & 0xff).to(torch.uint8)
    a[:, 8:12] = torch.tensor(list(bench.rank_ssrc(rank).to_bytes(4, "big")),
                              dtype=torch.uint8, device=dev)
    ln = torch.randint(12, 12 + payload + 1, (n,), dtype=torch.int32,
                       device=dev, generator=g)
    orig = a.clone()
    d = a.view(-1)
    off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    cap = torch.full((n,), slot, dtype=torch.int32, device=dev)
    st = torch.full((n,), -1, dtype=torch.int32, device=dev)
    assert sess.protect_device(d, off, ln, d, off, cap, st) == 0
    assert sess.prepass_stats() == (1, 0), sess.prepass_stats()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank),
             policy=json.dumps(pols[rank]), arena=orig.cpu().numpy().reshape(-1),
             off=off.cpu().numpy().astype(np.uint64),
             len=ln.cpu().numpy().astype(np.uint32), slot=slot,
             out=d.cpu().numpy(), status=st.cpu().numpy(),
             olen=cap.cpu().numpy().astype(np.uint32), how=how)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
