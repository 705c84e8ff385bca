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
KT_ADV = {"k_verify_groups": (90000.0, 9), "k_rs_sac": (85000.0, 1)}


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
               "roofline": bench.roofline_of(KT_ADV, {"k_verify_groups": {"k_verify_groups[1]": 100,
                                                                           "k_verify_groups[4]": 300}}, peak, None,
                                             "c5"),
               "kernel_avg_us": {k: v[0] for k, v in KT_ADV.items()}}
        cpu = None
        if rank == 0:
            th, machine, quota = bench.host_cores()
            cpu = bench.cpu_label({"value": 4000.0, "unit": "rounds/s", "kind": "port", "sample": "stub"}, th,
                                  machine, quota)
            rec["cpu_baseline"] = bench.cpu_label({"value": 30.0, "unit": "recovers/s", "sample": "stub"}, th,
                                                  machine, quota)
        head = {"value": 1e6 * 30 / dt, "n_gpus": world, "steps": 30, "warmup": 1, "ms_per_step": dt / 30 * 1e3,
                "scaling": "strong", "data": "stub", "config": {"workload": "stub", "global_rounds": 1000000},
                "batch_fallbacks": 0}
        tables = {"kernel_avg_us": {k: v[0] for k, v in KT.items()}, "peak": peak}
        line = bench.report(rank, world, head, roof, cpu, {"recover": rec, "adversarial": adv, "c1": None,
                                                           "live_latency": None, "sync": None}, tables, tables_out)
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
    assert len(line) < 4096, len(line)
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["roofline"]["frac"] > 0 and d["roofline"]["chip"]["frac"] > 0
    assert d["recover"]["value"] == 300000.0 and d["recover"]["roofline"]["frac"] > 0
    assert "kernel_avg_us" not in d["recover"] and "note" not in d["recover"]
    assert d["cpu_baseline"]["cores"] >= 1 and d["recover"]["cpu_baseline"]["value"] == 30.0
    side = json.load(open(out))
    assert side["recover"]["kernel_avg_us"]["k_rc_straus"] == 150000.0


def test_roofline_without_peak_reports_achieved():
    r = bench.roofline_of(KT_REC, {"k_rc_straus": 50000}, None, None, "c3")
    assert r["achieved"] > 0 and r["frac"] is None and r["issue_frac"] is None
