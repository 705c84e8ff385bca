"""bench.py's rank-dependent post-processing at world size 2 (gloo, stubbed timings): every value a rank
computes after the timed regions -- the max-over-ranks step time, the headline roofline, the Recover and
adversarial rooflines, the report -- must exist on every rank (a None that only exists off rank 0, such as a
peak measured on rank 0 alone, crashed the 8-GPU bench of round 2 before rank 0 printed), and rank 0's line
must stay under 4 KB with the headline and the Recover values in it."""
import json
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench

# a stub per-kernel timing table {name: (avg us, launches)} shaped like the real one
KT = {"k_exp_pm3d4": (1260.0, 12), "k_h2c_p1a": (230.0, 2), "k_h2c_p3": (420.0, 2), "k_dec_p1": (410.0, 2),
      "k_pair_miller_coop": (4300.0, 2), "k_final_coop": (2400.0, 2), "k_msm_aff_add": (210.0, 6)}
KT_REC = {"k_rc_straus": (150000.0, 1), "k_kmsm_chunks": (65000.0, 1), "k_exp_pm3d4": (6600.0, 6)}
KT_ADV = {"k_ck_miller": (56000.0, 3), "k_ck_expsq": (5300.0, 15), "k_ck_prep": (8300.0, 3), "k_rs_sac": (64000.0, 1)}
KT_NEG = {"k_exp_pm3d4": (1500.0, 40), "k_xq_sum": (900.0, 10), "k_xg_hlines": (3000.0, 30), "k_ck_miller": (4000.0, 30),
          "k_ck_expsq": (700.0, 150)}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, peaks, tables_out, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        peak = peaks[rank]
        dt = bench.max_over_ranks(0.30 + 0.01 * rank, world)
        roof = bench.headline_roofline(KT, KT, 125000, peak, 1000000, 30, world, dt)
        rec = {"metric": "Recover/s", "value": 300000.0, "unit": "recovers/s", "n_gpus": world,
               "roofline": bench.roofline_of(KT_REC, {"k_rc_straus": 50000}, peak, None, "c3"),
               "kernel_avg_us": {k: v[0] for k, v in KT_REC.items()}, "note": "x" * 500}
        adv = {"metric": "adversarial", "value": 7600.0, "unit": "recovers/s",
               "roofline": bench.pipeline_roofline(KT_ADV, {1: 345000, 4: 360000}, 10000, peak, None, "c5"),
               "kernel_avg_us": {k: v[0] for k, v in KT_ADV.items()}}
        neg = {"metric": "negative " * 20, "value": 5.1e6, "unit": "rounds/s", "steps": 10, "ms_per_step": 19.6,
               "corrupted_rounds": 1000, "batch_fallbacks": 10, "checks_per_batch": [6250.0, 3700.0, 4000.0],
               "isolation_kernel_share": 0.41,
               "roofline": bench.xr_roofline(KT_NEG, [62500, 37000, 40000], 250000, peak),
               "kernel_avg_us": {k: v[0] for k, v in KT_NEG.items()}, "note": "n" * 300}
        vpn = {"metric": "vp negative " * 10, "value": 3.1e6, "unit": "partials/s", "s_per_step": 0.8,
               "corrupted": 262000, "roofline": bench.pipeline_roofline(KT_ADV, {1: 900000, 4: 640000}, 10000, peak,
                                                                        None, "c5vp"),
               "kernel_avg_us": {k: v[0] for k, v in KT_ADV.items()}, "note": "v" * 200}
        cpu = None
        if rank == 0:
            th, machine, quota = bench.host_cores()
            cpu = bench.cpu_label({"value": 4000.0, "unit": "rounds/s", "kind": "port", "sample": "stub"}, th,
                                  machine, quota)
            rec["cpu_baseline"] = bench.cpu_label({"value": 30.0, "unit": "recovers/s", "sample": "stub"}, th,
                                                  machine, quota)
        head = {"value": 1e6 * 30 / dt, "n_gpus": world, "steps": 30, "warmup": 1, "ms_per_step": dt / 30 * 1e3,
                "scaling": "strong", "data": "synthetic linked chain data/chain_v1 (CPU-twin generated, seed tools/synthetic.py)",
                "config": {"workload": "w" * 230, "global_rounds": 1000000, "rounds_per_gpu": 100000,
                           "batches_per_gpu": 1, "hip_hw_queues": 16, "parallelism": "rounds sharded dp1"},
                "batch_fallbacks": 0}
        tables = {"kernel_avg_us": {k: v[0] for k, v in KT.items()}, "peak": peak}
        c2 = {"metric": "BASELINE configs[2]: VerifyPartial on all 64 shares of every round + Lagrange Recover " * 2,
              "value": 150000.0, "unit": "recovers/s", "value_recover_from_verdicts": 200000.0,
              "partials_verified_per_s": 1.3e7, "verify_partials_s": 0.5, "recover_s": 0.13,
              "recover_from_verdicts_s": 0.02, "note": "y" * 400,
              "roofline": bench.roofline_of(KT_REC, {"k_rc_straus": 50000}, peak, None, "c3vp")}
        c1 = {"metric": "C1: n=5 t=3, 5 Signs + Recover + VerifyRecovered per round (BASELINE configs[0])",
              "value": 13500.0, "unit": "rounds/s", "rounds": 1000, "s_per_step": 0.074, "note": "z" * 100}
        lat = {"recover_verified_ms": 11.783, "recover_full_ms": 27.938, "verify_recovered_ms": 10.879,
               "metric": "live-round latency, one round at n=64 t=33 (ms per call)"}
        syn = {"metric": "syncFrom catch-up rounds/s (bulk.sync_from, beacon/beacon.go:529-607)", "value": 523540.0,
               "unit": "rounds/s", "rounds": 100000, "batch": 25000, "s": 0.19101}
        if rank == 0:
            for x, v in ((c2, 40.0), (c1, 600.0)):
                x["cpu_baseline"] = bench.cpu_label({"value": v, "unit": "x/s", "kind": "port", "sample": "stub"}, th,
                                                    machine, quota)
        line = bench.report(rank, world, head, roof, cpu, {"recover": rec, "adversarial": adv, "c1": c1,
                                                           "live_latency": lat, "sync": syn, "c2_verify_all": c2,
                                                           "c2_negative": neg, "vp_negative": vpn},
                            tables, tables_out)
        q.put((rank, "ok", line))
    except Exception as e:  # noqa: BLE001 -- report any failure of any rank to the test
        q.put((rank, "error: %r" % (e,), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("peak1", ["measured", "missing"])
def test_bench_report_world2(tmp_path, peak1):
    world = 2
    peak0 = {"tmac_s": 39.0, "source": "stub", "clock_mhz": 2400.0}
    peaks = [peak0, dict(peak0) if peak1 == "measured" else None]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    out = str(tmp_path / "tables.json")
    ps = [ctx.Process(target=_worker, args=(r, world, port, peaks, out, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, status, line = q.get(timeout=120)
        res[r] = (status, line)
    for p in ps:
        p.join(timeout=60)
    assert res[0][0] == "ok" and res[1][0] == "ok", res
    assert res[1][1] is None  # only rank 0 prints
    line = res[0][1]
    print("line bytes", len(line))
    assert len(line) < 4608, len(line)  # the driver keeps the last 8 KB of the output
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["roofline"]["frac"] > 0 and d["roofline"]["chip"]["frac"] > 0
    assert d["recover"]["value"] == 300000.0 and d["recover"]["roofline"]["frac"] > 0
    assert d["c2_verify_all"]["value"] == 150000.0 and d["c2_verify_all"]["cpu_baseline"]["value"] == 40.0
    assert "kernel_avg_us" not in d["recover"] and "note" not in d["recover"]
    assert d["cpu_baseline"]["cores"] >= 1 and d["recover"]["cpu_baseline"]["value"] == 30.0
    assert d["c2_negative"]["value"] == 5.1e6 and d["c2_negative"]["roofline"]["frac"] > 0
    assert d["vp_negative"]["roofline"]["frac"] > 0 and d["adversarial"]["roofline"]["frac"] > 0
    side = json.load(open(out))
    assert side["recover"]["kernel_avg_us"]["k_rc_straus"] == 150000.0


def test_roofline_without_peak_reports_achieved():
    r = bench.roofline_of(KT_REC, {"k_rc_straus": 50000}, None, None, "c3")
    assert r["achieved"] > 0 and r["frac"] is None and r["issue_frac"] is None
