"""bench.py's reporting contract, on CPU (no GPU calls):

* the stdout line the driver parses stays small (round 2's 36 KB line, with
  the per-launch-shape PMC tables inline, was not parsed) and keeps the
  headline fields, `roofline` and `cpu_baseline`;
* `--gpus N` launches N rank processes when no outer launcher set WORLD_SIZE,
  and refuses a WORLD_SIZE that disagrees with it.
"""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADLINE = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")


def _full_report():
    """round 2's full bench output (profiles/r02_bench.json: every leg plus the
    28 KB `pmc` section), the worst case the line must fit"""
    with open(os.path.join(ROOT, "profiles", "r02_bench.json")) as f:
        return json.load(f)


def test_compact_line_fits_and_keeps_contract():
    out = _full_report()
    assert len(json.dumps(out)) > 30000  # the input really is the oversize case
    line = bench.compact(out)
    text = json.dumps(line, separators=(",", ":"))
    assert len(text) <= bench.LINE_MAX_BYTES
    assert "\n" not in text
    for k in HEADLINE:
        assert k in line, k
    rl = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rl, k
    assert rl["bound"] in ("hbm", "mfma")
    cb = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert line["commitment_verified"] is True
    assert "pmc" not in line
    # the per-kernel HBM summary survives in compact form
    assert isinstance(line.get("hbm_by_kernel"), dict) and line["hbm_by_kernel"]
    # the legs stay as summaries (not shed) at round 2's size
    for leg in ("sumcheck", "mle_open", "logup", "hyperplonk", "msm_strong_scaling"):
        assert isinstance(line[leg], dict), leg
    json.loads(text)


def test_compact_sheds_under_pressure():
    out = _full_report()
    out["hyperplonk"]["bulk"] = ["x" * 150] * 200  # a leg grows far past the budget
    line = bench.compact(out)
    assert len(json.dumps(line, separators=(",", ":"))) <= bench.LINE_MAX_BYTES
    for k in HEADLINE + ("roofline", "cpu_baseline"):
        assert k in line


def test_compact_rounds_floats():
    assert bench._sig(0.123456789) == 0.1235
    assert bench._sig(838000123.7) == 838000000.0
    assert bench._sig(True) is True and bench._sig(7) == 7
    assert bench._sig(float("nan")) is None


@pytest.mark.parametrize("gpus,env,want", [
    (1, {}, "run"),
    (8, {}, "launch"),
    (2, {"WORLD_SIZE": "2"}, "run"),
    (1, {"WORLD_SIZE": "1"}, "run"),
])
def test_launch_plan(gpus, env, want):
    assert bench.launch_plan(gpus, env) == want


def test_launch_plan_mismatch_is_an_error():
    r = bench.launch_plan(8, {"WORLD_SIZE": "4"})
    assert r not in ("run", "launch") and "WORLD_SIZE" in r
    assert bench.launch_plan(0, {}) not in ("run", "launch")


def test_launch_cmd_reruns_this_script_per_rank():
    cmd = bench.launch_cmd(4, ["--gpus", "4", "--steps", "3"], 29501)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert os.path.basename(cmd[-5]) == "bench.py"


def test_hbm_by_kernel_prefers_leg_keys():
    pmc = {"k_msm_accumulate": {"hbm_gbps": 1.0, "frac_hbm_peak": 0.1, "avg_us": 9.0,
                                "launches": 2},
           "k_msm_accumulate#probe_msm": {"hbm_gbps": 2.0, "frac_hbm_peak": 0.2, "avg_us": 16000.0,
                                          "launches": 1},
           "k_msm_accumulate#probe_mle": {"hbm_gbps": 3.0, "frac_hbm_peak": 0.3, "avg_us": 4000.0,
                                          "launches": 6},
           "k_msm_accumulate@1703936": {"hbm_gbps": 4.0, "frac_hbm_peak": 0.4, "avg_us": 1.0,
                                        "launches": 1}}
    hk = bench.hbm_by_kernel(pmc)
    assert set(hk) == {"k_msm_accumulate#probe_msm", "k_msm_accumulate#probe_mle"}
    assert list(hk)[0] == "k_msm_accumulate#probe_mle"  # 24 ms total before 16 ms
    assert bench._headline_traffic({"k_msm_accumulate#probe_msm": {
        "read_bytes_per_launch": 10.0, "write_bytes_per_launch": 2.0, "launches": 1}}) == 12.0


def test_setup_rank_orders_torch_then_library_comm(monkeypatch):
    """`bench.py --gpus 8`'s per-rank sequence (VERDICT r3 "next" 2): torch's
    RCCL process group on cuda:local_rank first, then the library context on
    the same device, then rank 0's ncclUniqueId broadcast through torch and
    qg_ctx_attach_comm with it."""
    import torch
    import torch.distributed as tdist
    calls = []
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: calls.append(("set_device", d)))
    monkeypatch.setattr(tdist, "init_process_group",
                        lambda backend, device_id=None: calls.append(("init", backend,
                                                                      str(device_id))))

    def bcast(obj, src=0):
        calls.append(("broadcast", obj[0], src))
        obj[0] = b"I" * 128

    monkeypatch.setattr(tdist, "broadcast_object_list", bcast)

    class FakeDevice:
        def __init__(self, d):
            calls.append(("ctx", d))
            self.world = 1

        @staticmethod
        def comm_unique_id():
            calls.append(("unique_id",))
            return b"I" * 128

        def attach_comm(self, rank, world, uid):
            calls.append(("attach", rank, world, uid == b"I" * 128))
            self.world = world

    class Q:
        Device = FakeDevice

    for rank, local in ((0, 0), (5, 5)):
        calls.clear()
        dev, dist = bench.setup_rank(Q, rank, 8, local)
        assert dist is tdist and dev.world == 8
        want = [("set_device", local), ("init", "nccl", f"cuda:{local}"), ("ctx", local)]
        want += [("unique_id",), ("broadcast", b"I" * 128, 0)] if rank == 0 else \
            [("broadcast", None, 0)]
        want += [("attach", rank, 8, True)]
        assert calls == want, calls
    calls.clear()
    dev, dist = bench.setup_rank(Q, 0, 1, 0)
    assert dist is None and calls == [("ctx", 0)]
