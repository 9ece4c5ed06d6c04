"""bench.py's host-side helpers (no GPU): the CPU-baseline thread count from
the cgroup quota, and the time-bounded reference legs."""
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cgroup_cpus_v2_and_v1(tmp_path):
    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    assert bench.cgroup_cpus(str(tmp_path)) == 16
    (tmp_path / "cpu.max").write_text("150000 100000\n")
    assert bench.cgroup_cpus(str(tmp_path)) == 2      # 1.5 CPUs -> 2 threads
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert bench.cgroup_cpus(str(tmp_path)) is None
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("800000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert bench.cgroup_cpus(str(v1)) == 8
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    assert bench.cgroup_cpus(str(v1)) is None
    assert bench.cgroup_cpus(str(tmp_path / "none")) is None


def test_bounded_leg_result_and_limit():
    lib = os.path.join(ROOT, "oracle", "_ref", "bench_ref_int.so")
    if not os.path.exists(lib):
        pytest.skip("oracle/_ref not built")
    r = bench._bounded("_ref_rate", lib, "protect", 160, False, 2, 0.5)
    assert r is not None and r[0] > 0 and r[1] > 0
    # a leg past its limit reports nothing instead of stalling the bench
    assert bench._bounded("_ref_rate", lib, "protect", 160, False, 2, 60.0,
                          limit=1) is None


def test_traffic_counts_read_requests_at_their_size():
    """roofline.traffic: 32/64/128-B read requests at their size plus
    WRITE_SIZE; gfx950's FETCH_SIZE (128-B requests at 64 B) stays a raw
    secondary figure, and a missing pass gives no number"""
    class A:
        op = "protect"
    pmc = {"TCC_EA0_RDREQ_32B_sum": 10.0, "TCC_EA0_RDREQ_64B_sum": 100.0,
           "TCC_EA0_RDREQ_128B_sum": 1000.0, "TCC_EA0_RDREQ_sum": 1110.0,
           "WRITE_SIZE": 200.0, "FETCH_SIZE": 70.0}
    rd = 32 * 10 + 64 * 100 + 128 * 1000
    assert bench.read_bytes(pmc) == rd
    assert bench.traffic_bytes(pmc) == rd + 200 * 1024
    sp = bench.traffic_split(A(), 100, 172, 10, pmc)
    assert sp["read_bytes"] == rd and sp["write_bytes"] == 200 * 1024
    assert sp["read_amplification"] == rd / (100 * 172)
    assert sp["write_amplification"] == 200 * 1024 / (100 * 182)
    assert sp["fetch_size_raw"] == 70 * 1024
    assert bench.traffic_bytes({"WRITE_SIZE": 1.0}) is None


def test_pmc_counter_sums_every_matching_kernel_per_step(tmp_path):
    """the key-bucket GCM form launches k_gcm_bk and k_gcm each step: the
    counter per step is both kernels' total over the steps, not the mean
    over all their dispatches"""
    rows = ["Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value"]
    d = 0
    for step in range(3):
        for name, v in (("k_gcm_bk<14, true>(GcmArgs)", 1000.0),
                        ("k_gcm<14, true, false, false>(GcmArgs)", 10.0),
                        ("k_pp_classify(...)", 5.0)):
            d += 1
            rows.append('%d,"%s",WRITE_SIZE,%s' % (d, name, v))
            rows.append('%d,"%s",SQ_WAVES,1' % (d, name))
    # a kernel of the warmup's first batch only: spread over the 3 steps
    d += 1
    rows.append('%d,"k_gcm<14, true, false, true>(GcmArgs)",WRITE_SIZE,300' % d)
    p = tmp_path / "counter_collection.csv"
    p.write_text("\n".join(rows) + "\n")
    assert bench.pmc_counter(str(p), ["k_gcm"], "WRITE_SIZE") == 1110.0
    assert bench.pmc_counter(str(p), ["k_icm"], "WRITE_SIZE") is None


def test_pmc_counter_takes_the_measured_direction(tmp_path):
    """an unprotect run's sender protects with the same kernels: only the
    direction measured counts (the PROTECT template argument)"""
    assert bench.kernel_protect(
        "void (anonymous namespace)::k_icm_hmac<10, true, false, 0, 0>"
        "(IcmArgs)") is False
    assert bench.kernel_protect("k_icm_stg<10, true, true>(IcmArgs)") is True
    assert bench.kernel_protect("k_gcm<14, false, true, false>(G)") is False
    assert bench.kernel_protect("k_gcm_bk<14, true>(GcmArgs)") is True
    assert bench.kernel_protect("k_pp_classify(ClassifyArgs)") is None
    rows = ["Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value"]
    for d in range(7):   # the sender's batches
        rows.append('%d,"k_gcm_bk<14, true>(GcmArgs)",WRITE_SIZE,500' % d)
    for d in range(7, 10):
        rows.append('%d,"k_gcm_bk<14, false>(GcmArgs)",WRITE_SIZE,400' % d)
    p = tmp_path / "counter_collection.csv"
    p.write_text("\n".join(rows) + "\n")
    assert bench.pmc_counter(str(p), ["k_gcm"], "WRITE_SIZE", False) == 400.0
    assert bench.pmc_counter(str(p), ["k_gcm"], "WRITE_SIZE", True) == 500.0
