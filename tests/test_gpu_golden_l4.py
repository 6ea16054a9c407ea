"""The GPU entry points against the golden vectors of the reference's own
checksum.cpp (tests/golden/l4/, made by tests/golden/gen_l4_golden.py from
/root/reference/checksum.cpp:8-36 compiled unchanged).

Compared with the fixtures directly — no oracle in between: wg_l4csum_desc
over every record under each descriptor kernel, wg_l4csum_uniform over the two
uniform PacketBatch runs, and wg_verify_desc over the well-formed records
(evaluate_packet's gates pass, csum_start = the IP header size): its L4 result
is calc_l4_checksum exactly when the TCP / UDP length floor lets the checksum
run (include/worker/evaluator.hpp:61,91), and L4_OK is set iff that result is 0.
"""
import json
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden" / "l4"
PKT_DESC = np.dtype([("offset", "<u8"), ("len", "<u4"), ("csum_start", "<u2"), ("flags", "u1"), ("rsvd", "u1")])


def _load(dev):
    import torch

    buf = np.fromfile(GOLD / "packets.bin", dtype=np.uint8)
    d = np.fromfile(GOLD / "desc.bin", dtype=PKT_DESC)
    kind = np.fromfile(GOLD / "kind.u8", dtype=np.uint8)
    exp = np.fromfile(GOLD / "expected.u16", dtype="<u2")
    man = json.loads((GOLD / "manifest.json").read_text())
    dbuf = torch.from_numpy(buf).to(dev)
    dd = torch.from_numpy(d.view(np.int64).reshape(-1, 2).copy()).to(dev)
    return buf, d, kind, exp, man, dbuf, dd


L4_VARIANTS = [{}, {"l4_coop": 0}, {"l4_coop": 0, "l4_small": 0}, {"l4_coop": 0, "l4_nt": 0}]


@pytest.mark.parametrize("knobs", L4_VARIANTS, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()) or "default")
def test_l4csum_desc_equals_reference(gpu, knobs):
    import torch

    import wireglider_amd as wga

    _, _, _, exp, _, dbuf, dd = _load(gpu)
    saved = {k: wga.tune_get(k) for k in knobs}
    try:
        for k, v in knobs.items():
            wga.tune_set(k, v)
        out = wga.calc_l4_checksum_desc(dbuf, dd)
        torch.cuda.synchronize()
    finally:
        for k, v in saved.items():
            wga.tune_set(k, v)
    np.testing.assert_array_equal(out.cpu().numpy(), exp)


def test_l4csum_uniform_runs_equal_reference(gpu):
    import torch

    import wireglider_amd as wga

    _, _, _, exp, man, dbuf, _ = _load(gpu)
    for run in man["uniform_runs"]:
        o, seg, cnt = run["offset"], run["segment_size"], run["count"]
        out = wga.calc_l4_checksum_batch(dbuf[o:o + seg * cnt], seg, bool(run["flags"] & 1), bool(run["flags"] & 2),
                                         run["csum_start"])
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), exp[run["first"]:run["first"] + cnt], err_msg=run["group"])


@pytest.mark.parametrize("vs", [None, 0, 6, 8])
def test_verify_desc_equals_reference(gpu, vs):
    import torch

    import wireglider_amd as wga

    _, d, kind, exp, _, dbuf, dd = _load(gpu)
    saved = wga.tune_get("verify_small")
    try:
        if vs is not None:
            wga.tune_set("verify_small", vs)
        verdict, l4 = wga.verify_desc(dbuf, dd)
        torch.cuda.synchronize()
    finally:
        wga.tune_set("verify_small", saved)
    verdict, l4 = verdict.cpu().numpy(), l4.cpu().numpy()
    well = (kind & 1) != 0
    v6, tcp = (d["flags"] & 1) != 0, (d["flags"] & 2) != 0
    ihs = np.where(v6, 40, 20)
    runs = (d["len"] - ihs) > np.where(tcp, 20, 8)  # the length floors let calc_l4_checksum run
    assert np.all(verdict[well] & 1)  # WG_VERDICT_IP_OK
    sel = well & runs
    np.testing.assert_array_equal(l4[sel], exp[sel])
    np.testing.assert_array_equal((verdict[sel] & 2) != 0, exp[sel] == 0)
    assert np.all(l4[well & ~runs] == 0) and np.all((verdict[well & ~runs] & 2) == 0)
    assert sel.sum() >= 150 and np.count_nonzero(exp[sel] == 0) >= 60
