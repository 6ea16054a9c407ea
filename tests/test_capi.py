"""The C-ABI library loads, exports every symbol include/wireglider_amd.h
declares, and the C++ drop-in header (include/wireglider/checksum.hpp)
compiles with a plain host compiler and reproduces the reference test oracle.
No compute calls: these run without a GPU."""
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
HDR = ROOT / "include" / "wireglider_amd.h"


def declared_symbols():
    txt = HDR.read_text()
    return sorted(set(re.findall(r"^(?:int|uint64_t|const char \*)\s*(wg_\w+)\(", txt, flags=re.M)))


def test_header_declares_expected():
    syms = declared_symbols()
    import wireglider_amd as wga

    assert syms == sorted(wga.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    import wireglider_amd as wga

    out = subprocess.run(["nm", "-D", "--defined-only", str(wga.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    for s in declared_symbols():
        assert s in exported, s
    # the C++ drop-in symbol with the reference's mangled signature
    # uint16_t wireglider::calc_l4_checksum(std::span<const uint8_t>, bool, bool, uint16_t)
    assert "_ZN10wireglider16calc_l4_checksumESt4spanIKhLm18446744073709551615EEbbt" in exported


def test_abi_and_device_count():
    import wireglider_amd as wga

    assert wga.lib.wg_abi_version() == wga.ABI_VERSION == 2
    assert wga.lib.wg_strerror(-1) == b"invalid argument"
    assert wga.device_count() >= 0


def test_no_oracle_in_product():
    # the product library never links or loads the oracle
    import wireglider_amd as wga

    out = subprocess.run(["nm", "-D", str(wga.LIB_PATH)], capture_output=True, text=True, check=True).stdout
    assert "orc_" not in out
    assert "oracle" not in (ROOT / "wireglider_amd" / "__init__.py").read_text().split('"""')[2]


def test_invalid_args_rejected_without_gpu():
    import wireglider_amd as wga

    # validated on the host before any HIP call
    assert wga.lib.wg_l4csum_uniform(None, 100, 1500, 20, 0, None, None) == -1
    assert wga.lib.wg_l4csum_uniform(1, 100, 0, 20, 0, 1, None) == -1
    assert wga.lib.wg_l4csum_desc(16, 17, 1, 16, None) == -1
    # the kernel-shaped read probe takes segments of at most 2 KiB
    assert wga.lib.wg_probe_read(16, 1 << 20, 16, 1, 4096, None) == -1
    assert wga.lib.wg_probe_read(16, 100, 16, 1, 1500, None) == -1
    # AEAD batches: segment size 0 / past 64 KiB, no key, misaligned or missing outputs
    key = bytes(32)
    assert wga.lib.wg_aead_encrypt_batch(16, 100, 0, key, 1, 0, 16, None, None) == -1
    assert wga.lib.wg_aead_encrypt_batch(16, 100, 65536, key, 1, 0, 16, None, None) == -1
    assert wga.lib.wg_aead_encrypt_batch(16, 100, 50, None, 1, 0, 16, None, None) == -1
    assert wga.lib.wg_aead_encrypt_batch(16, 100, 50, key, 1, 0, 17, None, None) == -1  # out not 16-B aligned
    assert wga.lib.wg_aead_decrypt_batch(16, 100, 64, key, 16, None, None) == -1  # status required
    assert wga.lib.wg_aead_decrypt_verify_batch(16, 100, 64, key, 16, 16, None, 16, None) == -1  # verdict required
    assert wga.lib.wg_aead_decrypt_verify_batch(16, 100, 64, key, 16, 16, 16, None, None) == -1  # l4 required
    assert wga.lib.wg_aead_decrypt_verify_batch(16, 100, 65536 + 33, key, 16, 16, 16, 16, None) == -1
    assert wga.lib.wg_aead_decrypt_verify_batch(16, 0, 64, key, 16, 16, 16, 16, None) == 0  # empty batch: no-op
    # encap: bounds, too many super-buffers, misaligned message buffer, no-op on n = 0
    assert wga.lib.wg_encap_encrypt(16, 16, 16, 16, 1, key, 1, 0, 16, 1 << 16, 0, 1500, 16, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_encrypt(16, 16, 16, 16, 1, key, 1, 0, 16, 1 << 16, 45, 0, 16, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_encrypt(16, 16, 16, 16, 1, key, 1, 0, 16, 1 << 16, 45, 70000, 16, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_encrypt(16, 16, 16, 16, (1 << 20) + 1, key, 1, 0, 16, 1 << 16, 45, 1500, 16, 16, 16, None,
                                    None) == -1
    assert wga.lib.wg_encap_encrypt(16, 16, 16, 16, 1, key, 1, 0, 16, 1 << 16, 45, 1500, 8, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_encrypt(16, 16, 16, 16, 1, None, 1, 0, 16, 1 << 16, 45, 1500, 16, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_encrypt(16, 16, 16, 16, 0, key, 1, 0, 16, 1 << 16, 45, 1500, 16, 16, 16, None, None) == 0
    # 2^32 messages or more in one call: the 32-bit counter scan would wrap
    # (repeated nonces), so it is refused on the host
    assert wga.lib.wg_encap_encrypt(16, 16, 16, 16, 1 << 20, key, 1, 0, 16, 1 << 16, 4096, 1500, 16, 16, 16, None,
                                    None) == -1
    assert wga.lib.wg_encap_batch(16, 16, 1 << 20, 16, 16, key, 1, 0, 16, 1 << 16, 4096, 1500, 16, 16, 16, None,
                                  None) == -1
    # the fused encap step: the same bounds, out (the header slots) required
    assert wga.lib.wg_encap_batch(16, 16, 1, 16, 16, key, 1, 0, 16, 1 << 16, 0, 1500, 16, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_batch(16, 16, 1, 16, 16, key, 1, 0, 16, 1 << 16, 45, 70000, 16, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_batch(16, 16, 1, None, 16, key, 1, 0, 16, 1 << 16, 45, 1500, 16, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_batch(16, 16, 1, 16, 16, key, 1, 0, 16, 1 << 16, 45, 1500, 8, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_batch(16, 16, 1, 16, 16, None, 1, 0, 16, 1 << 16, 45, 1500, 16, 16, 16, None, None) == -1
    assert wga.lib.wg_encap_batch(16, 16, (1 << 20) + 1, 16, 16, key, 1, 0, 16, 1 << 16, 45, 1500, 16, 16, 16, None,
                                  None) == -1
    assert wga.lib.wg_encap_batch(16, 16, 0, 16, 16, key, 1, 0, 16, 1 << 16, 45, 1500, 16, 16, 16, None, None) == 0


DROPIN_TEST = r"""
#include <cstdio>
#include <vector>
#include "wireglider/checksum.hpp"
int main(int argc, char **argv) {
    // argv[1]: create_packet_65536.bin, argv[2]: ref1_random_1_1500.u16, argv[3]: ref1_carry_1_63.u16
    std::vector<uint8_t> s(65536);
    std::vector<uint16_t> g(1500), c(63);
    FILE *f = fopen(argv[1], "rb"); size_t k = fread(s.data(), 1, s.size(), f); fclose(f);
    f = fopen(argv[2], "rb"); k += fread(g.data(), 2, g.size(), f); fclose(f);
    f = fopen(argv[3], "rb"); k += fread(c.data(), 2, c.size(), f); fclose(f);
    if (k != 65536 + 1500 + 63) return 2;
    int bad = 0;
    for (size_t n = 1; n <= 1500; n++)
        bad += wireglider::checksum(std::span<const uint8_t>(s.data(), n), 0) != g[n - 1];
    for (size_t n = 1; n <= 63; n++) {
        std::vector<uint8_t> p(n, 0xff); p[n - 1] = 1;
        bad += wireglider::checksum(p, 0) != c[n - 1];
    }
    // fixed extents (tests/test-checksum.cpp:27-51)
    using namespace wireglider::checksum_impl;
    std::span<const uint8_t> d(s.data(), 16);
    auto ref = [&](size_t o, size_t n) { return wireglider::checksum(d.subspan(o, n), 0); };
    bad += fold_complement(checksum_nofold(d.subspan<0, 1>(), 0)) != ref(0, 1);
    bad += fold_complement(checksum_nofold(d.subspan<0, 2>(), 0)) != ref(0, 2);
    bad += fold_complement(checksum_nofold(d.subspan<0, 4>(), 0)) != ref(0, 4);
    bad += fold_complement(checksum_nofold(d.subspan<0, 8>(), 0)) != ref(0, 8);
    bad += fold_complement(checksum_nofold(d.subspan<0, 16>(), 0)) != ref(0, 16);
    // pseudo header: in_addr-sized overload and span overload agree
    uint32_t a = 0x0100a8c0, b = 0x0200a8c0;
    auto p1 = wireglider::pseudo_header_checksum<uint32_t>(17, a, b, 1480);
    // (the span overload is ambiguous with an lvalue span exactly as in the
    // reference's overload set; call the nofold form like checksum.cpp does)
    auto p2 = fold_complement(pseudo_header_checksum_nofold(17, std::span<const uint8_t, 4>((const uint8_t *)&a, 4),
                                                            std::span<const uint8_t, 4>((const uint8_t *)&b, 4), 1480));
    bad += p1 != p2;
    printf("%d %u\n", bad, (unsigned)p1);
    return bad != 0;
}
"""


def test_dropin_header_compiles_and_matches_reference(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(DROPIN_TEST)
    exe = tmp_path / "t"
    subprocess.run(["g++", "-std=c++20", "-O2", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)], check=True)
    g = ROOT / "tests" / "golden" / "ref"
    r = subprocess.run([str(exe), str(g / "create_packet_65536.bin"), str(g / "ref1_random_1_1500.u16"),
                        str(g / "ref1_carry_1_63.u16")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    bad, p1 = r.stdout.split()
    # cross-check the pseudo-header value against the oracle
    import oracle

    src_b = np.array([0xC0, 0xA8, 0x00, 0x01], np.uint8)
    dst_b = np.array([0xC0, 0xA8, 0x00, 0x02], np.uint8)
    exp = oracle.lib.orc_fold_complement(
        oracle.lib.orc_pseudo_header_nofold(17, src_b.ctypes.data, dst_b.ctypes.data, 4, 1480))
    assert int(p1) == exp


def test_tune_knobs_validate_and_round_trip():
    """wg_tune_set / wg_tune_get (host only): every documented key round
    trips, out-of-range values are rejected and leave the knob unchanged."""
    import wireglider_amd as wga

    keys = re.findall(r'^ \*   "(\w+)"', HDR.read_text(), flags=re.M)
    assert {"l4_nt", "gso_groups", "verify_small", "l4_small", "host_d2h", "gso_ablate"} <= set(keys)
    # round 4 removed the rejected variants' knobs: no longer accepted
    for gone in ("l4_ppw", "l4_occ", "l4_descv", "l4_iters", "l4_split_waves", "verify_dm", "verify_occ",
                 "verify_hdr", "verify_wblk", "gro_lds", "gro_wide", "gro_chunks", "gro_iters", "aead_pair",
                 "aead_flex"):
        assert gone not in keys
        with pytest.raises(Exception):
            wga.tune_get(gone)
    for k in keys:
        v = wga.tune_get(k)
        wga.tune_set(k, v)
        assert wga.tune_get(k) == v
    for k, bad in (("l4_small", 1), ("l4_small", 4), ("verify_small", 3), ("l4_small_uniform", 1),
                   ("gso_groups", 0), ("gso_groups", 65),
                   ("gso_waves", 16), ("gso_ablate", 7), ("gso_ablate", 2), ("l4_coop_waves", 3),
                   ("l4_coop_waves", 32), ("aead_k", 1), ("aead_k", 4)):
        v = wga.tune_get(k)
        with pytest.raises(Exception):
            wga.tune_set(k, bad)
        assert wga.tune_get(k) == v
    # the library ships no wrong-output variant (round-1 gso_ablate = 2 removed)
    assert wga.lib.wg_tune_set(b"gso_ablate", 2) == -1
    with pytest.raises(Exception):
        wga.tune_get("no_such_knob")
    v = wga.tune_get("l4_nt")
    wga.tune_set("l4_nt", 0)  # zero is a value, not "unset"
    assert wga.tune_get("l4_nt") == 0
    wga.tune_set("l4_nt", v)


def test_tune_environment_overrides():
    """WG_<KEY> is read once with the same validation: a valid value
    (including 0) overrides the default, an invalid one is ignored."""
    import os
    import sys

    code = ("import wireglider_amd as w; print(w.tune_get('l4_nt'), w.tune_get('gso_groups'), "
            "w.tune_get('l4_small'), w.tune_get('verify_small'))")
    code += "; print(w.tune_get('gso_ablate'))"
    env = dict(os.environ, WG_L4_NT="0", WG_GSO_GROUPS="5", WG_L4_SMALL="3", WG_VERIFY_SMALL="0x8", WG_GSO_ABLATE="2")
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True, check=True)
    nt, groups, small, vs, abl = map(int, out.stdout.split())
    assert (nt, groups, vs) == (0, 5, 8)
    assert abl == 0  # WG_GSO_ABLATE=2 is not an accepted value: ignored
    assert small == 5  # 3 is not an accepted value: default kept


def test_bench_valu_issue_checks_kernel_symbol():
    """bench.py prices the AEAD line against a committed VALU instruction
    count only when that profile counted the kernel the line times: the
    symbol launch_aead picks (aead_kernel_symbol mirrors its K / group rule)."""
    import bench
    import wireglider_amd as wga

    assert bench.aead_kernel_symbol(wga, 1500) == \
        "void wg::aead_kernel<0, 3, false, false, 0, true, false>(wg::AeadParams)"
    assert bench.aead_kernel_symbol(wga, 64) == "void wg::aead_kernel<1, 2, false, false, 0, false, false>(wg::AeadParams)"
    assert bench.aead_kernel_symbol(wga, 9000, True, True).startswith("void wg::aead_kernel<64, 2, true, true, 0, false,")
    # wg_encap_batch: the header-synthesizing instantiation (encap_synth = 1, the default)
    assert bench.aead_kernel_symbol(wga, 1500, gso=2) == \
        "void wg::aead_kernel<0, 3, false, false, 2, true, true>(wg::AeadParams)"
    assert bench.aead_kernel_symbol(wga, 1500, gso=1).endswith("1, true, false>(wg::AeadParams)")
    # exact-size groups always fit: 32 lanes, 2 packets per wave, 4 x 2 x (32 + 6,080) B
    assert bench.aead_kernel_symbol(wga, 6070).endswith("false, false, 0, true, false>(wg::AeadParams)")
    saved = {k: wga.tune_get(k) for k in ("aead_stage", "encap_synth")}
    try:
        wga.tune_set("aead_stage", 0)
        assert bench.aead_kernel_symbol(wga, 1500).endswith("0, false, false>(wg::AeadParams)")
        assert bench.aead_kernel_symbol(wga, 1500, gso=2).endswith("2, false, false>(wg::AeadParams)")
        wga.tune_set("aead_stage", 1)
        wga.tune_set("encap_synth", 0)
        assert bench.aead_kernel_symbol(wga, 1500, gso=2).endswith("2, true, false>(wg::AeadParams)")
    finally:
        for k, v in saved.items():
            wga.tune_set(k, v)
    prof = {"kernel": "void wg::aead_kernel<0, 3, false, true>(wg::AeadParams)", "valu_winst_per_launch": 8e8}
    ok = bench.valu_issue(dict(prof, kernel="K"), "K", 1.0, "aead")
    assert ok["valu_issue"]["frac"] == round(8e8 / 1e-3 / bench.VALU_PEAK_WINST, 4)
    assert "valu_issue_refused" in bench.valu_issue(prof, "K", 1.0, "aead")
    assert bench.valu_issue(None, "K", 1.0, "aead") == {}
