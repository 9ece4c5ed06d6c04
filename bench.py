#!/usr/bin/env python3
"""bench.py -- device-resident srtp_protect() throughput on MI355X.

Workload (BASELINE.json configs[1], the headline): AES-128-ICM + HMAC-SHA1-80
protect, one stream (SSRC 0xcafebabe), 2^20 packets x 1400-byte payload
(1412-byte RTP packets -> 1422-byte SRTP packets) resident in HBM.  One step
= srtp_protect_device() over the whole batch: header parse, the in-order
index / replay / key-limit pre-pass, and the HIP crypto kernels, in place.
Every step gets its own batch (the sender's next W+K batches: the same
packets with the 16-bit sequence numbers advanced, as a sender would
produce them; replay protection rejects a repeated index), all built in HBM
before the timed region.

--op unprotect: the receive side of the same workload -- the batches are
protected (untimed) by a sender session, and one step is
srtp_unprotect_device() over one batch, in place, on the receiver session.
--reorder P / --dup Q (unprotect): the receive batches arrive in network
order -- a fraction P of arrivals swapped with one up to 32 places later,
a fraction Q replaced by a copy of a packet up to 64 places earlier
(replay_fail) -- built in HBM before the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W]
                  [--config icm128|gcm256|g711] [--op protect|unprotect]
                  [--reorder P] [--dup Q]

Multi-GPU: one process per GPU (torch.distributed.run, nccl = RCCL), each
rank protects its own 2^20-packet batch of its own stream (weak scaling).
Rank 0 creates the session and the others receive a replica through the
library's C ABI (srtp_mi355x_session_broadcast: one ncclBroadcast of the
exported session over xGMI on torch's own communicator; under gloo the
exported blob goes through the process group); the data path has no
collective.  SRTP_BENCH_DEVICE=d puts every rank on device d (the N > 1
path on a one-GPU box, with SRTP_DIST_BACKEND=gloo).  value =
all ranks' packets / max rank time.  `--gpus N` with N > 1 and no
WORLD_SIZE in the environment starts the N ranks itself (a
torch.distributed.run child, before this process touches the GPU) and exits
with its status; under a launcher WORLD_SIZE must equal N.
BASELINE configs[4] (AES-256-GCM, 8M x 1400 B over 8 x MI355X, RCCL key
broadcast) is `python bench.py --config gcm256 --gpus 8`: 2^20 packets per
rank, 8 ranks.

--dry-run: the same orchestration (rank launch, barrier-bracketed timing,
max over ranks, the one JSON line) over gloo on the CPU with a stub step
(rank r sleeps (r + 1) ms), for tests without a GPU.

Extra fields: roofline (dominant kernel, HIP-event timed on the stream the
kernels ran on; `traffic` = the L2's 32/64/128-B fabric read requests at
their size + WRITE_SIZE per launch from separate rocprofv3 PMC passes,
`traffic_over_algorithmic` = that over the algorithmic bytes,
`traffic_split` = read and write amplification separately, `issue` = VALU / LDS instruction floors, `additive_frac`
their sum over the launch), cpu_baseline (the reference, cisco/libsrtp built from
its own sources, srtp_protect() per packet on host threads, rank 0 only).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (cipher policy dict, payload bytes, packets per GPU, tag bytes)
    # g711 = BASELINE configs[3]: 64k SSRC streams, a distinct master key per
    # stream (SURVEY §8d "primary"), packets round-robin over the streams
    "icm128": (dict(cipher_type=1, cipher_key_len=30, auth_type=3,
                    auth_key_len=20, auth_tag_len=10, sec_serv=3), 1400,
               1 << 20, 10),
    "gcm256": (dict(cipher_type=7, cipher_key_len=44, auth_type=0,
                    auth_key_len=0, auth_tag_len=16, sec_serv=3), 1400,
               1 << 20, 16),
    "g711": (dict(cipher_type=1, cipher_key_len=30, auth_type=3,
                  auth_key_len=20, auth_tag_len=10, sec_serv=3), 160,
             1 << 23, 10),
    # configs[3]'s shape under AES-256-GCM-16 (not a BASELINE config: the
    # many-stream GCM forms, e.g. --template's one key for 64k clones)
    "g711gcm": (dict(cipher_type=7, cipher_key_len=44, auth_type=0,
                     auth_key_len=0, auth_tag_len=16, sec_serv=3), 160,
                1 << 23, 16),
}
WORKLOAD = {
    "icm128": "AES-128-ICM + HMAC-SHA1-80 {op}, 1M packets x 1400B, 1 stream",
    "gcm256": "AES-256-GCM-16 {op}, 1M packets x 1400B per GPU, 1 stream",
    "g711": "AES-128-ICM + HMAC-SHA1-80 {op}, 8M packets x 160B, "
            "64k SSRC streams (distinct keys, round-robin)",
    "g711gcm": "AES-256-GCM-16 {op}, 8M packets x 160B, 64k SSRC streams "
               "(distinct keys, round-robin)",
}


def workload(a):
    """config.workload: the configuration and the operation timed"""
    if a.template:
        return ("{c} {op}, 8M packets x 160B, 64k SSRC "
                "streams under ONE template key (ssrc_any_outbound / "
                "_inbound; streams created on the device by the warmup's "
                "first batch)").format(
                    op=a.op, c="AES-256-GCM-16" if a.config == "g711gcm"
                    else "AES-128-ICM + HMAC-SHA1-80")
    return WORKLOAD[a.config].format(op=a.op)


# master key: test/srtp_driver.c test_key (46 bytes) -- any key works
TEST_KEY = ("e1f97a0d3e018be0d64fa32c06de41390ec675ad498afeebb6960b3aabe6"
            "c173c317f2dabe357793b6960b3aabe6")
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
STREAMS = {"icm128": 1, "gcm256": 1, "g711": 65536, "g711gcm": 65536}
# (config, multi-GPU) -> the BASELINE.json configs[] entry the line measures
BASELINE_CONFIG = {("icm128", False): 1, ("gcm256", False): 2,
                   ("g711", False): 3, ("gcm256", True): 4}


def stream_keys(n, seed=0x5352545030303031):
    """distinct 46-byte master keys (hex) from splitmix64, one per stream"""
    out, x = [], seed
    for _ in range(n):
        b = bytearray()
        while len(b) < 46:
            x = (x + 0x9e3779b97f4a7c15) & (2**64 - 1)
            z = x
            z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & (2**64 - 1)
            z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & (2**64 - 1)
            b += (z ^ (z >> 31)).to_bytes(8, "little")
        out.append(bytes(b[:46]).hex())
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE or 1")
    ap.add_argument("--dry-run", action="store_true",
                    help="gloo on the CPU with a stub step (no GPU)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="icm128", choices=sorted(CONFIGS))
    ap.add_argument("--op", default="protect", choices=["protect", "unprotect"])
    ap.add_argument("--packets", type=int, default=0,
                    help="override packets per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipelined", action="store_true",
                    help="protect through srtp_protect_device_async: the "
                    "next batch is submitted while the previous one's "
                    "kernel runs (kernel_ms then comes from the warmup "
                    "launches, which run synchronously with timing on)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="target wall time of the CPU-baseline sample")
    ap.add_argument("--reorder", type=float, default=0.0,
                    help="--op unprotect: fraction of arrivals swapped with "
                    "one up to 32 places later (network reordering)")
    ap.add_argument("--dup", type=float, default=0.0,
                    help="--op unprotect: fraction of arrivals that are a "
                    "copy of a packet up to 64 places earlier (duplicates; "
                    "the packet they displace is lost): replay_fail")
    ap.add_argument("--template", action="store_true",
                    help="--config g711 / g711gcm only: the 64k SSRCs "
                    "under one "
                    "template policy (ssrc_any_outbound sender, "
                    "ssrc_any_inbound receiver) instead of 64k specific "
                    "streams with distinct keys (SURVEY 8(d) configs[3] "
                    "variant); the first warmup batch creates the streams")
    ap.add_argument("--percall", action="store_true",
                    help="the drop-in per-call path instead: one 1400-B "
                    "packet per srtp_protect() / srtp_unprotect() call "
                    "(tools/percall_bench, srtp_driver.c:1202-1268's loop), "
                    "next to the reference's per-call time on one host core")
    ap.add_argument("--percall-calls", type=int, default=100000)
    ap.add_argument("--traffic", default="auto", choices=["auto", "off"],
                    help="auto: measure roofline.traffic and roofline.issue "
                         "with rocprofv3 PMC passes (child processes, N=1 "
                         "only)")
    return ap.parse_args()


def note(msg):
    """progress on stderr (stdout carries only the JSON line): a GPU box
    takes a run that writes nothing for minutes to be hung"""
    print("bench: " + msg, file=sys.stderr, flush=True)


# where each crypto kernel's PROTECT template argument sits
_DIR_ARG = {"k_icm_hmac": 2, "k_icm_stg": 2, "k_gcm": 1, "k_gcm_bk": 1}


def kernel_protect(name):
    """True / False from a crypto kernel's demangled name (its PROTECT
    template argument), None when the name carries none"""
    import re
    m = re.search(r"(k_icm_hmac|k_icm_stg|k_gcm_bk|k_gcm)<([^>]*)>", name)
    if not m:
        return None
    args = [x.strip() for x in m.group(2).split(",")]
    i = _DIR_ARG[m.group(1)]
    return args[i] == "true" if i < len(args) else None


def pmc_counter(path, kernels, counter, protect=None):
    """one rocprofv3 --pmc counter per step of the crypto launches: the
    total over every kernel whose name contains one of `kernels`
    (substrings) divided by the launches of the most frequent of them -- one
    per step (k_gcm matches both launches of the key-bucket form, k_gcm_bk
    and k_gcm; a kernel of the warmup's first batch only is spread over the
    steps instead of counted as if it ran in each).  protect: only the
    kernels of that direction (an unprotect run's sender protects its
    inputs with the same kernels)"""
    import csv
    tot, disp = {}, {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name", "") != counter:
                continue
            name = row.get("Kernel_Name", "")
            if protect is not None and kernel_protect(name) not in (None,
                                                                    protect):
                continue
            if any(k in name for k in kernels):
                tot[name] = tot.get(name, 0.0) + float(
                    row.get("Counter_Value", 0) or 0)
                disp.setdefault(name, set()).add(row.get("Dispatch_Id"))
    if not disp:
        return None
    return sum(tot.values()) / max(len(d) for d in disp.values())


# PMC passes (MI355X_MICROARCH.md: one pass holds at most 4 TCC counters,
# FETCH_SIZE takes 3 and WRITE_SIZE 2, so they run separately).  The read
# bytes come from the L2's memory-side read requests by size: gfx950's
# FETCH_SIZE tallies a 128-byte request at 64 B (MI355X_MICROARCH.md:298),
# so it is kept only as a raw secondary figure.
RDREQ = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
         "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_sum")
PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE",), RDREQ,
              ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAVES"))


def read_bytes(pmc):
    """bytes the L2 requested from the fabric per launch: 32 / 64 / 128-B
    read requests at their size (None without the request-size pass)"""
    if any(c not in pmc for c in RDREQ[:3]):
        return None
    return (32.0 * pmc[RDREQ[0]] + 64.0 * pmc[RDREQ[1]] +
            128.0 * pmc[RDREQ[2]])


def traffic_bytes(pmc):
    """roofline.traffic: read requests at their size + WRITE_SIZE (exact for
    streaming stores, MI355X_MICROARCH.md:299); None if a pass is missing"""
    rd = read_bytes(pmc)
    if rd is None or "WRITE_SIZE" not in pmc:
        return None
    return rd + pmc["WRITE_SIZE"] * 1024.0


DIST_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
             "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE",
             "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
             "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS",
             "SRTP_FORCE_DIST")


def traffic_split(a, n, rtp_len, tag, pmc):
    """read and write bytes per launch, each against the algorithmic bytes
    of its direction (read / write amplification), the request counts they
    come from, and FETCH_SIZE as counted (raw, 128-B requests at half).
    The counters see the L2's fabric requests, Infinity-Cache hits included
    (MI355X_MICROARCH.md:297): re-read key records served on-die count."""
    rd_alg = n * (rtp_len + (tag if a.op == "unprotect" else 0))
    wr_alg = n * (rtp_len + (0 if a.op == "unprotect" else tag))
    rd = read_bytes(pmc)
    w = pmc["WRITE_SIZE"] * 1024.0 if "WRITE_SIZE" in pmc else None
    if rd is None and w is None:
        return None
    out = {"read_bytes": rd, "write_bytes": w,
           "read_algorithmic": rd_alg, "write_algorithmic": wr_alg,
           "read_amplification": rd / rd_alg if rd is not None else None,
           "write_amplification": w / wr_alg if w is not None else None,
           "rdreq": {k.replace("TCC_EA0_", "").replace("_sum", ""): pmc[k]
                     for k in RDREQ if k in pmc}}
    if "FETCH_SIZE" in pmc:
        out["fetch_size_raw"] = pmc["FETCH_SIZE"] * 1024.0
    return out


def measure_pmc(a, kernels, device=0):
    """per-launch PMC counters of the dominant kernel over a short run of
    this same workload, one rocprofv3 --pmc pass per entry of PMC_PASSES,
    each a child process started before this process touches the GPU.
    `traffic` is the read requests at their size plus WRITE_SIZE
    (traffic_bytes(); traffic_split() per direction)."""
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return {}
    base = tempfile.mkdtemp(prefix="srtp_pmc_", dir="/tmp")
    got = {}
    for k, ctrs in enumerate(PMC_PASSES):
        note("PMC pass %d/%d: %s" % (k + 1, len(PMC_PASSES), " ".join(ctrs)))
        d = os.path.join(base, "p%d" % k)
        cmd = [prof, "--pmc"] + list(ctrs) + [
               "--output-format", "csv", "-d", d, "-o",
               "p", "--", sys.executable, os.path.abspath(__file__),
               "--config", a.config, "--op", a.op, "--steps", "2",
               "--warmup", "1",
               "--no-cpu-baseline", "--traffic", "off"]
        if a.template:
            cmd.append("--template")
        if a.packets:
            cmd += ["--packets", str(a.packets)]
        # a one-rank child on this rank's device (at N > 1 rank 0 measures
        # before the process group forms; the other ranks wait in it)
        env = {k: v for k, v in os.environ.items() if k not in DIST_VARS}
        env.update(TMPDIR="/tmp", SRTP_BENCH_DEVICE=str(device))
        try:
            # the child's stderr (its progress notes) stays visible
            subprocess.run(cmd, stdout=subprocess.DEVNULL, timeout=150,
                           env=env)
        except subprocess.TimeoutExpired:
            break
        csvs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                         recursive=True)
        if not csvs:
            break
        for c in ctrs:
            v = pmc_counter(csvs[0], kernels, c, a.op == "protect")
            if v is not None:
                got[c] = v
    shutil.rmtree(base, ignore_errors=True)
    return got


# issue floors measured on MI355X by probes (tools/valu_rate.hip,
# tools/lds_rate.hip): the fastest VALU wave-instruction
# (xor / and / add / bitop3) per SIMD, and one conflict-free ds_read_b32
# per CU
VALU_NS_PER_SIMD = 1.10
LDS_NS_PER_CU = 1.21
SIMDS, CUS = 1024, 256


def issue_roofline(pmc, kernel_ms):
    """SURVEY §8(d)'s second ceiling: the kernel's VALU and LDS
    wave-instructions (PMC) against the probe-measured issue floors"""
    v, l = pmc.get("SQ_INSTS_VALU"), pmc.get("SQ_INSTS_LDS")
    if v is None or l is None:
        return None
    fv = v * VALU_NS_PER_SIMD / SIMDS * 1e-6      # ms
    fl = l * LDS_NS_PER_CU / CUS * 1e-6
    # profiles/r04_icm_wavespec.md §6: an LDS read stream and a VALU stream
    # on one SIMD add up almost linearly, so the floor the kernel can reach
    # is their SUM (additive_frac, the headline); max_frac (the larger floor
    # alone) is kept as a secondary figure
    return {"bound": "valu+lds issue", "valu_insts": v, "lds_insts": l,
            "valu_floor_ms": fv, "lds_floor_ms": fl,
            "additive_frac": (fv + fl) / kernel_ms,
            "frac": (fv + fl) / kernel_ms,
            "max_frac": max(fv, fl) / kernel_ms,
            "valu_ns_per_simd": VALU_NS_PER_SIMD,
            "lds_ns_per_cu": LDS_NS_PER_CU}


def rank_ssrc(rank):
    """each rank protects its own stream (weak scaling, no shared state)"""
    return 0xcafebabe ^ rank


def timed_steps(step, steps, warmup, world, sync=None):
    """W untimed warmup steps, then K timed steps bracketed by a barrier and
    a device synchronize on both sides; returns (seconds, per-step results)
    with seconds = the MAX over ranks (gloo all_reduce)."""
    import torch.distributed as dist
    sync = sync or (lambda: None)
    # a process group of one rank (SRTP_FORCE_DIST=1) takes the same path
    on = world > 1 or (dist.is_available() and dist.is_initialized())
    for _ in range(warmup):
        step()
    sync()
    if on:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    res = [step() for _ in range(steps)]
    sync()
    if on:
        dist.barrier()
    dt = time.perf_counter() - t0
    if on:
        import torch
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
    return dt, res


# the one-GPU box's host share: gpurun grants 16 CPUs of a larger host
# (os.cpu_count() shows the whole host there)
HOST_SHARE = 16


def _bounded(fn, *args, limit=120):
    """bench.<fn>(*args) in a child process with a time limit (the parent
    has initialised the GPU, so the child is a fresh interpreter, not a
    fork); None when it fails or runs past the limit"""
    import subprocess
    code = ("import json, sys; sys.path.insert(0, %r); import bench; "
            "print(json.dumps(bench.%s(*json.loads(sys.argv[1]))))"
            % (ROOT, fn))
    try:
        r = subprocess.run([sys.executable, "-c", code, json.dumps(args)],
                           capture_output=True, text=True, timeout=limit)
        return tuple(json.loads(r.stdout.strip().splitlines()[-1]))
    except (subprocess.TimeoutExpired, ValueError, IndexError, TypeError):
        note("cpu baseline %s%r: no result within %d s" % (fn, args, limit))
        return None


def cgroup_cpus(root="/sys/fs/cgroup"):
    """the cgroup CPU quota in whole CPUs (cgroup v2 cpu.max or v1
    cfs_quota_us / cfs_period_us), None when there is none"""
    import math
    try:
        with open(os.path.join(root, "cpu.max")) as f:
            q, p = f.read().split()[:2]
        if q != "max":
            return max(1, math.ceil(int(q) / int(p)))
        return None
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(root, "cpu", "cpu.cfs_quota_us")) as f:
            q = int(f.read())
        with open(os.path.join(root, "cpu", "cpu.cfs_period_us")) as f:
            p = int(f.read())
        return max(1, math.ceil(q / p)) if q > 0 else None
    except (OSError, ValueError):
        return None


def _ref_rate(lib_path, op, payload, gcm, threads, seconds):
    """packets/s of the reference build at lib_path: calibrate with all
    `threads` threads on a short run, timing the whole call (unprotect's
    untimed protect pass and any lock contention between the threads
    included: a one-thread calibration sent OpenSSL unprotect at 16 threads
    past the child's time limit), then a run of ~`seconds` wall time"""
    L = C.CDLL(lib_path)
    fn = L.ref_bench if op == "protect" else L.ref_bench_unprotect
    fn.argtypes = [C.c_int, C.c_long, C.c_int, C.c_int, C.POINTER(C.c_double)]
    secs = C.c_double()
    cal = 1024
    while True:   # grow the calibration until its fixed costs are small
        t0 = time.perf_counter()
        fn(threads, cal, payload, int(gcm), C.byref(secs))
        wall = time.perf_counter() - t0
        if wall >= seconds / 8 or cal >= 1 << 22:
            break
        cal *= 4
    per_thread = max(cal, int(cal * seconds / max(wall, 1e-6)))
    done = fn(threads, per_thread, payload, int(gcm), C.byref(secs))
    return done / secs.value, done


def _ref_rate_streams(lib_path, payload, nstreams, threads, cycles=1):
    """the reference with nstreams specific-SSRC streams per srtp_t, packets
    round-robin (BASELINE configs[3]; every srtp_protect() scans the
    reference's stream list): `cycles` passes over the streams per thread
    (one pass of 65,536 packets per thread takes ~10-30 s of linear scans)"""
    L = C.CDLL(lib_path)
    fn = L.ref_bench_streams
    fn.argtypes = [C.c_int, C.c_long, C.c_int, C.c_int, C.POINTER(C.c_double)]
    secs = C.c_double()
    done = fn(threads, cycles * nstreams, payload, nstreams, C.byref(secs))
    if done <= 0 or secs.value <= 0:
        return None
    return done / secs.value, done


def _ref_rate_template(lib_path, payload, nstreams, threads, cycles=2,
                       op="protect", gcm=False):
    """the reference with ONE ssrc_any_outbound template per srtp_t and
    packets round-robin over nstreams SSRCs: the first pass clones every
    stream (srtp.c:2540-2559), later ones scan the cloned list; unprotect:
    one ssrc_any_inbound srtp_t per thread receiving a template sender's
    packets (clones on first authentication, srtp.c:3117-3155); gcm: the
    template policy is AES-256-GCM-16"""
    L = C.CDLL(lib_path)
    fn = L.ref_bench_template_policy
    fn.argtypes = [C.c_int, C.c_long, C.c_int, C.c_int, C.c_int, C.c_int,
                   C.POINTER(C.c_double)]
    secs = C.c_double()
    done = fn(threads, cycles * nstreams, payload, nstreams,
              int(op != "protect"), int(gcm), C.byref(secs))
    if done <= 0 or secs.value <= 0:
        return None
    return done / secs.value, done


def cpu_baseline_template(payload, nstreams, op="protect", gcm=False):
    """--template: the reference's own template path (oracle/bench_ref.c
    ref_bench_template / ref_bench_template_unprotect), both crypto
    backends, the faster one as value"""
    ref = os.path.join(ROOT, "oracle", "_ref")
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    th = max(1, min(HOST_SHARE, affinity, quota or affinity))
    res = {}
    # (the built-in crypto kernel has no AES-GCM)
    for k in ("ossl",) if gcm else ("ossl", "int"):
        path = os.path.join(ref, "bench_ref_%s.so" % k)
        if not os.path.exists(path):
            continue
        note("cpu baseline %s template path, %d SSRCs, %d threads"
             % (k, nstreams, th))
        r = _bounded("_ref_rate_template", path, payload, nstreams, th, 2, op,
                     gcm, limit=240)
        if r:
            res[k] = r
    if not res:
        return None
    mk = max(res, key=lambda k: res[k][0])
    backend = {"ossl": "OpenSSL 3 crypto backend",
               "int": "built-in crypto kernel"}
    return {"value": res[mk][0], "unit": "pkt/s", "cores": th,
            "kind": "reference",
            "sample": "%d x srtp_%s(), one ssrc_any_%s %stemplate "
                      "per srtp_t, %d SSRCs round-robin (first pass clones "
                      "them), %d threads, cisco/libsrtp 3.0.0 with the %s, "
                      "built from source (oracle/Makefile.ref)"
                      % (res[mk][1], op,
                         "outbound" if op == "protect" else "inbound",
                         "AES-256-GCM-16 " if gcm else "",
                         nstreams, th, backend[mk]),
            "backends": {"openssl": res["ossl"][0] if "ossl" in res else None,
                         "internal_kernel": res["int"][0] if "int" in res
                         else None}}


def cpu_baseline(cfg, op, payload, seconds):
    """The reference on the host: srtp_protect() (or srtp_unprotect()) per
    packet, one srtp_t per thread (oracle/bench_ref.c over
    oracle/_ref/bench_ref_*.so, cisco/libsrtp built from its own sources).
    Both crypto backends are timed (`backends`): OpenSSL 3 and the built-in
    crypto kernel that north_star names (no AES-GCM); `value` is the faster
    of the two for this workload.  Timed at every CPU this process may run
    on (`value_affinity`; the sample sized for the HOST_SHARE CPUs the
    one-GPU box grants) and at 16 threads (`value_16`); `value` / `cores` is
    the faster of the two.  configs[3]
    (g711) adds `many_ssrc`: the reference with its 65,536 streams in one
    srtp_t, packets round-robin -- its own stream lookup is a linear scan
    (srtp/srtp.c:5292-5305)."""
    gcm = cfg in ("gcm256", "g711gcm")
    ref = os.path.join(ROOT, "oracle", "_ref")
    ossl = os.path.join(ref, "bench_ref_ossl.so")
    intk = os.path.join(ref, "bench_ref_int.so")
    affinity = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    # the CPUs this process can actually use: its affinity mask, capped by
    # its cgroup's CPU quota (the one-GPU box shows the whole host's 256
    # CPUs in the mask and grants a 16-CPU quota; 256 threads on that quota
    # collapse OpenSSL 3 into lock contention)
    threads = max(1, min(256, affinity, quota or affinity))
    call = "srtp_%s()" % op
    res, res16 = {}, {}
    for k, path in (("ossl", ossl), ("int", intk)):
        if not os.path.exists(path) or (k == "int" and gcm):
            continue
        note("cpu baseline %s, %d threads" % (k, threads))
        r = _bounded("_ref_rate", path, op, payload, gcm, threads, seconds)
        if threads != 16:
            note("cpu baseline %s, 16 threads" % k)
            r16 = _bounded("_ref_rate", path, op, payload, gcm, 16,
                           seconds / 2)
        else:
            r16 = r
        if r:
            res[k] = r
        if r16:
            res16[k] = r16
    if not res or not res16:
        return None
    # `value` is the faster backend (the stronger baseline: OpenSSL wins on
    # large payloads, the built-in kernel on small ones, where OpenSSL's
    # per-call EVP setup dominates); both are listed
    main_key = max(res, key=lambda k: res[k][0])
    backend = {"ossl": "OpenSSL 3 crypto backend",
               "int": "built-in crypto kernel"}
    rate, done = res[main_key]
    k16 = max(res16, key=lambda k: res16[k][0])
    # the stronger of the two thread counts is `value` (the one-GPU box
    # grants 16 CPUs; more threads than that only share them)
    best = (rate, done, threads, main_key)
    if res16[k16][0] > rate:
        best = (res16[k16][0], res16[k16][1], 16, k16)
    out = {"value": best[0], "unit": "pkt/s", "cores": best[2],
           "kind": "reference",
           "sample": "%d x %s of %d-byte payloads, %d threads x 1 srtp_t, "
                     "cisco/libsrtp 3.0.0 with the %s, built from source "
                     "(oracle/Makefile.ref)" % (best[1], call, payload,
                                                 best[2], backend[best[3]]),
           "payload_GBps": best[0] * payload / 1e9,
           "value_affinity": rate, "threads_affinity": threads,
           "value_16": res16[k16][0],
           "host_cpus": os.cpu_count(), "affinity_cpus": affinity,
           "cgroup_cpus": quota,
           "backends": {"openssl": res["ossl"][0] if "ossl" in res else None,
                        "internal_kernel": res["int"][0] if "int" in res
                        else None}}
    if gcm:
        out["backends"]["internal_kernel_note"] = "no AES-GCM in that kernel"
    if cfg == "g711" and op == "protect":
        ms = {}
        th = min(threads, HOST_SHARE)   # 65,536 stream contexts per thread
        for k, path in (("ossl", ossl), ("int", intk)):
            note("cpu baseline %s, %d streams per srtp_t, %d threads"
                 % (k, STREAMS[cfg], th))
            r = _bounded("_ref_rate_streams", path, payload, STREAMS[cfg], th) \
                if os.path.exists(path) else None
            if r:
                ms[k] = r
        if ms:
            mk = max(ms, key=lambda k: ms[k][0])
            out["many_ssrc"] = {
                "value": ms[mk][0], "unit": "pkt/s", "threads": th,
                "backend": backend[mk],
                "sample": "%d x srtp_protect(), %d streams with distinct keys "
                          "per srtp_t, round-robin" % (ms[mk][1], STREAMS[cfg]),
                "backends": {"openssl": ms["ossl"][0] if "ossl" in ms else None,
                             "internal_kernel": ms["int"][0] if "int" in ms
                             else None}}
    return out


def distribute_keys(keys_hex, world, dev):
    """Session (re)key: rank 0's master keys reach every rank in ONE
    broadcast of the key blob -- RCCL over xGMI with the nccl backend (gloo
    on CPU tensors in the tests).  Every rank then derives its session keys
    from them (srtp_create runs the KDF), so nothing else is exchanged and
    the data path has no collective."""
    import torch
    import torch.distributed as dist
    raw = b"".join(bytes.fromhex(k) for k in keys_hex)
    blob = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    if world > 1 or (dist.is_available() and dist.is_initialized()):
        dist.broadcast(blob, src=0)
    raw = blob.cpu().numpy().tobytes()
    w = len(raw) // len(keys_hex)
    return [raw[i * w:(i + 1) * w].hex() for i in range(len(keys_hex))]


def replicate_session(L, policies, world, rank, dev, backend):
    """Session replication (north_star "RCCL broadcast of
    session keys over xGMI"): rank 0 creates the session -- its KDF derives
    the session keys on its GPU -- and every other rank receives a replica
    (streams, derived key records, stream state) through the library's C
    ABI.  With RCCL (backend nccl) that is srtp_mi355x_session_broadcast on
    torch's own communicator: ncclBroadcast of the exported blob from device
    memory over xGMI.  Otherwise (gloo, or no communicator handle) the
    exported blob (srtp_mi355x_session_export) goes through the process
    group and srtp_mi355x_session_import rebuilds it.  Returns (session,
    how)."""
    import torch
    import torch.distributed as dist
    on = world > 1 or (dist.is_available() and dist.is_initialized())
    if not on:
        return L.Session(policies), "none (one rank)"
    sess = L.Session(policies) if rank == 0 else None
    tdev = dev if backend == "nccl" else torch.device("cpu")
    comm = None
    if backend == "nccl":
        try:
            dist.barrier()   # the communicator exists after a collective
            pg = dist.distributed_c10d._get_default_group()
            comm = pg._get_backend(torch.device("cuda", dev.index))._comm_ptr()
        except Exception as e:   # noqa: BLE001 - torch-version dependent
            note("no RCCL communicator handle (%s): blob over the group" % e)
            comm = None
    # every rank takes the same path
    ok = torch.tensor([1 if comm else 0], dtype=torch.int32, device=tdev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok[0]):
        stream = torch.cuda.current_stream().cuda_stream
        return (L.session_broadcast(sess, comm, 0, stream),
                "srtp_mi355x_session_broadcast (ncclBroadcast on the "
                "process group's RCCL communicator)")
    blob = sess.export_blob() if rank == 0 else b""
    n = torch.tensor([len(blob)], dtype=torch.int64, device=tdev)
    dist.broadcast(n, src=0)
    if rank == 0:
        buf = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(tdev)
    else:
        buf = torch.empty(int(n[0]), dtype=torch.uint8, device=tdev)
    dist.broadcast(buf, src=0)
    how = ("srtp_mi355x_session_export / _import, blob broadcast over %s"
           % backend)
    if rank == 0:
        return sess, how
    return L.Session.from_blob(buf.cpu().numpy().tobytes()), how


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a, argv):
    """--gpus N > 1 without a launcher: run torch.distributed.run as a
    CHILD process (this process has not touched the GPU and never execs),
    one rank per GPU on this node; rank 0's JSON line reaches our stdout
    through the inherited descriptor.  Returns the child's exit status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % a.gpus, "--master-addr=127.0.0.1",
           "--master-port=%d" % _free_port(), os.path.abspath(__file__)]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd + list(argv), env=env)


def resolve_world(a):
    """(world, rank, local rank); --gpus must agree with a launcher's
    WORLD_SIZE"""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus is None:
        a.gpus = world
    if a.gpus != world:
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%d" % (a.gpus, world))
    return (world, int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def run_percall(a, json_out):
    """--percall: an unchanged libsrtp caller's shape -- every packet its
    own srtp_protect() / srtp_unprotect() call, i.e. a GPU batch of one --
    timed in C (tools/percall_bench, a child process), for AES-128-ICM +
    HMAC-SHA1-80 and AES-256-GCM-16; the cpu_baseline leg times the
    reference's own per-packet call on ONE host core (oracle/_ref, the
    internal crypto kernel for AES-ICM, OpenSSL for AES-GCM)"""
    import subprocess
    exe = os.path.join(ROOT, "tools", "percall_bench")
    if not os.path.exists(exe):
        raise SystemExit("bench: tools/percall_bench not built "
                         "(make -C libsrtp_amd percall)")
    res, cpu = {}, {}
    ref = os.path.join(ROOT, "oracle", "_ref")
    for c, gcm, lib in (("icm128", False, "bench_ref_int.so"),
                        ("gcm256", True, "bench_ref_ossl.so")):
        note("per-call %s: %d calls per op" % (c, a.percall_calls))
        r = subprocess.run([exe, str(a.percall_calls), "gcm" if gcm else "icm"],
                           capture_output=True, text=True, timeout=600)
        if r.returncode:
            raise SystemExit("bench: percall_bench failed: " + r.stderr[-400:])
        res[c] = json.loads(r.stdout.strip().splitlines()[-1])
        path = os.path.join(ref, lib)
        if a.no_cpu_baseline or not os.path.exists(path):
            continue
        for op in ("protect", "unprotect"):
            note("cpu baseline per call: %s %s, 1 thread" % (c, op))
            rr = _bounded("_ref_rate", path, op, 1400, gcm, 1, 4.0)
            if rr:
                cpu["%s_%s_us_per_call" % (c, op)] = 1e6 / rr[0]
    out = {"metric": "per-call latency of srtp_protect() / srtp_unprotect(), "
                     "one 1412-B RTP packet per call (drop-in path)",
           "value": res["icm128"]["protect_calls_per_s"], "unit": "calls/s",
           "higher_is_better": True, "n_gpus": 1, "dtype": "u8",
           "data": "synthetic (one reused packet, seq advanced per call)",
           "config": {"workload": "srtp_driver.c srtp_bits_per_second loop: "
                      "%d calls per op, 1400-B payload" % a.percall_calls},
           "percall": {c: {k: v for k, v in d.items()
                           if k.endswith(("_us_per_call", "_calls_per_s"))}
                       for c, d in res.items()},
           "cpu_baseline": {"kind": "reference", "cores": 1,
                            "sample": "srtp_protect()/srtp_unprotect() per "
                                      "packet, 1400-B payload, one thread "
                                      "(oracle/_ref)", **cpu}}
    print(json.dumps(out), file=json_out, flush=True)


def dry_run(a, world, rank, json_out):
    """the multi-rank orchestration without a GPU: gloo process group, a
    stub step that takes (rank + 1) ms, the same timing and JSON line"""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    pol, payload, npk, tag = CONFIGS[a.config]
    n = a.packets or npk

    def step():
        time.sleep(1e-3 * (rank + 1))
        return 0.0

    dt, _ = timed_steps(step, a.steps, a.warmup, world)
    if rank == 0:
        rec = result_line(a, world, n, payload, tag, dt, None, None, None)
        rec["dry_run"] = True
        print(json.dumps(rec), file=json_out, flush=True)
    if world > 1:
        dist.destroy_process_group()


def arrival_rows(n, reorder, dup, seed):
    """arrival order of a receive batch (the rows of the sent batch): local
    swaps of up to 32 places, then duplicates -- a copy of a packet that
    arrived up to 64 places earlier, in place of a packet that is lost"""
    import numpy as np
    rng = np.random.default_rng(seed)
    rows = np.arange(n, dtype=np.int64)
    for i in np.nonzero(rng.random(n) < reorder)[0]:
        j = min(n - 1, int(i) + int(rng.integers(1, 33)))
        rows[i], rows[j] = rows[j], rows[i]
    pos = np.nonzero(rng.random(n) < dup)[0]
    pos = pos[pos >= 64]
    isdup = np.zeros(n, dtype=bool)
    isdup[pos] = True
    for i in pos:
        src = int(i) - int(rng.integers(1, 65))
        while isdup[src]:
            src -= 1
        rows[i] = rows[src]
    return rows, len(pos)


def result_line(a, world, n, payload, tag, dt, roofline, cpu, prepass):
    rtp_len = 12 + payload
    value = n * a.steps * world / dt
    return {
        "metric": "SRTP packets/sec + payload GB/s, device-resident, "
                  "1M×1400B batch",
        "op": a.op,
        "value": value,
        "unit": "pkt/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (random payloads, seq advanced per step)",
        "config": {"workload": workload(a), "packets_per_gpu": n,
                   "packets_total": n * world,
                   "streams_per_gpu": STREAMS[a.config],
                   "payload_bytes": payload, "rtp_bytes": rtp_len,
                   "srtp_bytes": rtp_len + tag, "parallelism": "dp%d" % world,
                   "baseline_config": BASELINE_CONFIG.get(
                       (a.config, world > 1), None),
                   "submission": "pipelined (srtp_protect_device_async)"
                   if a.pipelined and a.op == "protect"
                   else "synchronous (srtp_%s_device)" % a.op,
                   **({"arrival": {"reorder": a.reorder, "dup": a.dup}}
                      if a.reorder or a.dup else {})},
        "payload_GBps": value * payload / 1e9,
        "roofline": roofline,
        "cpu_baseline": cpu,
        "prepass": prepass,
    }


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        sys.exit(launch_ranks(a, sys.argv[1:]))
    world, rank, local = resolve_world(a)
    if a.template and a.config not in ("g711", "g711gcm"):
        raise SystemExit("bench: --template applies to --config g711 / "
                         "g711gcm")
    # stdout carries exactly the one JSON line: native libraries' banners
    # (RCCL prints its version block at communicator init) go to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if a.dry_run:
        dry_run(a, world, rank, json_out)
        return
    if a.percall:
        run_percall(a, json_out)
        return
    try:
        run_gpu(a, world, rank, local, json_out)
    finally:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.destroy_process_group()


def run_gpu(a, world, rank, local, json_out):
    pol, payload, npk, tag = CONFIGS[a.config]
    kname = "k_gcm" if a.config in ("gcm256", "g711gcm") else "k_icm_hmac"
    kernels = (kname,)
    if a.config == "g711" and os.environ.get("SRTP_ICM_STG", "1") != "0":
        # configs[3]'s fused batches: the LDS-staged kernel, then the
        # per-lane form over the groups it listed (one launch per step each;
        # DESIGN.md §4 k_icm_stg); the HIP events bracket both
        kname = "k_icm_stg + k_icm_hmac (list pass)"
        kernels = ("k_icm_stg", "k_icm_hmac")
    # PMC passes first: child processes, before this one touches the GPU
    # SRTP_BENCH_DEVICE: every rank of this process on that device (the
    # N > 1 path exercised on a one-GPU box, with gloo: RCCL refuses two
    # ranks on one device)
    devno = int(os.environ.get("SRTP_BENCH_DEVICE", local))
    pmc = {}
    if rank == 0 and a.traffic == "auto":
        pmc = measure_pmc(a, kernels, devno)
    traffic = traffic_bytes(pmc)
    import torch
    import torch.distributed as dist
    # SRTP_FORCE_DIST=1: a one-rank process group, so the RCCL barrier,
    # key broadcast and max-over-ranks reduction run on a one-GPU box too
    backend = None
    torch.cuda.set_device(devno)
    if world > 1 or os.environ.get("SRTP_FORCE_DIST") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("SRTP_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group(backend,
                                    device_id=torch.device("cuda", devno))
        else:
            dist.init_process_group(backend)
    import libsrtp_amd as L
    dev = torch.device("cuda", torch.cuda.current_device())

    n = a.packets or npk
    nstreams = STREAMS[a.config]
    ssrc = rank_ssrc(rank)
    if nstreams == 1:
        # one stream per rank (SSRC-affine shards): rank 0's
        # session holds every rank's stream; each rank keeps its own shard
        # of the replica
        policies = [dict(pol, ssrc_type=1, ssrc=rank_ssrc(r), window_size=128,
                         allow_repeat_tx=0, keys=[TEST_KEY])
                    for r in range(world)]
        note("session: %d streams (GPU KDF on rank 0), replicated"
             % len(policies))
        sess, replication = replicate_session(L, policies, world, rank, dev,
                                              backend)
        for r in range(world):
            if r != rank and sess.remove_stream(rank_ssrc(r)) != 0:
                raise RuntimeError("bench: removing stream of rank %d" % r)
    elif a.template:
        # one template policy per rank (the same key everywhere): every
        # rank's first batch creates its 64k streams on its own GPU
        base = (0x10000000 + (rank << 20)) & 0xffffffff
        policies = [dict(pol, ssrc_type=3, ssrc=0, window_size=128,
                         allow_repeat_tx=0, keys=[TEST_KEY])]
        note("session: one template policy, %d SSRCs per batch" % nstreams)
        sess = L.Session(policies)
        replication = "template policy per rank" if backend else \
            "none (one rank)"
    else:
        # 64k streams per rank: the master keys (rank 0's) are broadcast and
        # every rank derives its own streams' session keys
        keys = distribute_keys(stream_keys(nstreams), world,
                               dev if backend == "nccl" else "cpu")
        base = (0x10000000 + (rank << 20)) & 0xffffffff
        policies = [dict(pol, ssrc_type=1, ssrc=base + k, window_size=128,
                         allow_repeat_tx=0, keys=[key])
                    for k, key in enumerate(keys)]
        note("session: %d streams (GPU KDF)" % len(policies))
        sess = L.Session(policies)
        replication = "master keys broadcast, KDF per rank" \
            if backend else "none (one rank)"

    note("building %d batches of %d packets in HBM" % (a.warmup + a.steps, n))
    # packet arenas in HBM, one per step: slot = roundup16(rtp_len + tag)
    rtp_len = 12 + payload
    slot = (rtp_len + tag + 15) & ~15
    nb = a.warmup + a.steps
    if nb * n * slot > (200 << 30):
        raise SystemExit("bench: %d batches x %d B do not fit the 200 GiB "
                         "arena budget" % (nb, n * slot))
    g = torch.Generator(device=dev).manual_seed(0x5352545030303031 & 0x7fffffff)
    base_arena = torch.randint(0, 256, (n, slot), dtype=torch.uint8,
                               device=dev, generator=g)
    base_arena[:, 0] = 0x80
    base_arena[:, 1] = 96
    base_arena[:, 4:8] = 0
    idx = torch.arange(n, dtype=torch.int64, device=dev)
    if nstreams == 1:
        base_arena[:, 8:12] = torch.tensor(list(ssrc.to_bytes(4, "big")),
                                           dtype=torch.uint8, device=dev)
    else:
        pk_ssrc = base + idx % nstreams         # round-robin over streams
        for k in range(4):
            base_arena[:, 8 + k] = ((pk_ssrc >> (24 - 8 * k)) & 0xff).to(
                torch.uint8)
    pk_seq = idx // nstreams                     # per-stream packet number
    per_stream = (n + nstreams - 1) // nstreams
    arenas = []
    for k in range(nb):
        ar = base_arena.clone()
        seq = (pk_seq + 0x1234 + k * per_stream) & 0xffff
        ar[:, 2] = (seq >> 8).to(torch.uint8)
        ar[:, 3] = (seq & 0xff).to(torch.uint8)
        arenas.append(ar.view(-1))
    del base_arena
    off = torch.arange(n, dtype=torch.int64, device=dev) * slot
    in_len = torch.full((n,), rtp_len, dtype=torch.int32, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    # one status array per batch, preset to a value no status takes, so the
    # check after the timed region sees every step's verdicts (a batch that
    # never ran keeps the preset)
    statuses = [torch.full((n,), -1, dtype=torch.int32, device=dev)
                for _ in range(nb)]
    stream = torch.cuda.current_stream().cuda_stream
    expect_dups = []
    if (a.reorder or a.dup) and a.op != "unprotect":
        raise SystemExit("--reorder / --dup apply to --op unprotect")
    if a.op == "unprotect":
        # the sender's side, untimed: protect every batch in place; the
        # receiver (`sess`) then unprotects them in order
        snd = L.Session([dict(p, ssrc_type=3 if a.template else 1)
                         for p in policies])
        if a.template:
            sess.close()
            sess = L.Session([dict(p, ssrc_type=2) for p in policies])
        srtp_len = torch.empty(n, dtype=torch.int32, device=dev)
        for ar in arenas:
            srtp_len.fill_(slot)
            if snd.protect_device(ar, off, in_len, ar, off, srtp_len,
                                  status, stream=stream) != 0 or \
                    int((status != 0).sum()):
                raise RuntimeError("bench: protecting the receive batches")
        snd.close()
        in_len = srtp_len
        if a.reorder or a.dup:
            # network arrival order, built untimed: each receive batch's
            # packets permuted (and duplicated) in HBM
            for k in range(nb):
                rows, ndup = arrival_rows(n, a.reorder, a.dup, 1000 + k)
                arenas[k] = arenas[k].view(n, slot)[
                    torch.from_numpy(rows).to(dev)].reshape(-1)
                expect_dups.append(ndup)
    sess.set_timing(True)
    # out_len: capacities in, lengths out -- one array per batch, each
    # packet's capacity its whole slot (what a caller with a slotted arena
    # passes), set before the timed region
    caps = [torch.full((n,), slot, dtype=torch.int32, device=dev)
            for _ in range(nb)]
    torch.cuda.synchronize()
    k_step = [0]
    fn = sess.protect_prepared if a.op == "protect" else \
        sess.unprotect_prepared
    # one descriptor per batch, built before the timed region
    descs = [sess.prepare_device(ar, off, in_len, ar, off, cp, st,
                                 stream=stream)
             for ar, cp, st in zip(arenas, caps, statuses)]

    pipelined = a.pipelined and a.op == "protect"
    warm_ms = []

    def step():
        b = descs[k_step[0]]
        k_step[0] += 1
        if pipelined and k_step[0] > a.warmup:
            if k_step[0] == a.warmup + 1:
                sess.set_timing(False)   # timing would synchronise
            st = sess.protect_prepared_async(b)
        else:
            st = fn(b)
        if st != 0:
            raise RuntimeError("srtp_%s_device: %s" % (a.op, st))
        if pipelined and k_step[0] <= a.warmup:
            warm_ms.append(sess.last_kernel_ms())
        return None if pipelined else sess.last_kernel_ms()

    dev_b0, host_b0 = sess.prepass_stats()
    note("%d warmup + %d timed steps" % (a.warmup, a.steps))
    dt, kms = timed_steps(step, a.steps, a.warmup, world,
                          sync=torch.cuda.synchronize)
    note("timed steps done: %.3f ms per step" % (dt * 1e3 / a.steps))
    if pipelined:
        # the warmup launches, synchronous with timing on; the first one
        # also pays the cold start, so it is left out when there are more
        if not warm_ms:
            raise SystemExit("--pipelined needs --warmup >= 1 (kernel timing)")
        kms = warm_ms[1:] or warm_ms
    if expect_dups:
        # every displaced copy is replay_fail (status 9), all else accepted
        bad = sum(int(((st != 0) & (st != 9)).sum()) +
                  abs(int((st == 9).sum()) - d)
                  for st, d in zip(statuses, expect_dups))
    else:
        bad = sum(int((st != 0).sum()) for st in statuses)
    dev_b, host_b = sess.prepass_stats()
    if bad or host_b != host_b0:
        raise SystemExit("bench: %d packets with a nonzero status, %d batches "
                         "on the host path" % (bad, host_b - host_b0))
    kernel_ms = sum(kms) / len(kms)
    algo_bytes = n * (rtp_len + rtp_len + tag)   # rtp + srtp, read + write
    achieved = algo_bytes / (kernel_ms * 1e-3) / 1e9
    if rank != 0:
        if backend:
            dist.barrier()   # rank 0's CPU baseline and line, then teardown
        return
    cpu = None
    if not a.no_cpu_baseline:
        # the host cores beside rank 0's GPU, after the timed region
        cpu = cpu_baseline_template(payload, nstreams, a.op,
                                    a.config == "g711gcm") if a.template else \
            cpu_baseline(a.config, a.op, payload, a.cpu_seconds)
    roofline = {"bound": "hbm", "achieved": achieved,
                "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_over_algorithmic":
                    traffic / algo_bytes if traffic else None,
                "traffic_split": traffic_split(a, n, rtp_len, tag, pmc),
                "kernel": kname, "kernel_ms": kernel_ms,
                "algorithmic_bytes_per_launch": algo_bytes,
                "issue": issue_roofline(pmc, kernel_ms)}
    prepass = {"device_batches": dev_b - dev_b0,
               "host_batches": host_b - host_b0,
               "last_abort": sess.prepass_last_abort()}
    out = result_line(a, world, n, payload, tag, dt, roofline, cpu, prepass)
    out["session_replication"] = replication
    print(json.dumps(out), file=json_out, flush=True)
    if backend:
        dist.barrier()


if __name__ == "__main__":
    main()
