#!/usr/bin/env python3
"""Generate the AEAD golden vectors with an INDEPENDENT
implementation: the system OpenSSL's libcrypto (3.0), through its public EVP
API by ctypes.  The reference's AEAD is libsodium's
crypto_aead_chacha20poly1305_ietf (proto/proto.cpp:507-516, 574-583;
un-vendored, Makefile:107-109), i.e. RFC 8439; OpenSSL's
EVP_chacha20_poly1305 implements the same RFC.

Also checks the RFC 8439 published test vectors (§2.3.2 block function,
§2.5.2 Poly1305, §2.8.2 AEAD) against OpenSSL before writing them, so each
committed vector is confirmed by two sources.  Output: aead_golden.json
(hex), consumed by tests/test_oracle_aead.py and tests/test_gpu_aead.py.
Run here (needs libcrypto.so.3); the GPU box only reads the JSON.
"""
import ctypes
import json
import random
from pathlib import Path

HERE = Path(__file__).resolve().parent
crypto = ctypes.CDLL("libcrypto.so.3")
vp, cp, ci = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int
crypto.EVP_CIPHER_CTX_new.restype = vp
crypto.EVP_chacha20_poly1305.restype = vp
crypto.EVP_chacha20.restype = vp
for f in ("EVP_EncryptInit_ex", "EVP_EncryptUpdate", "EVP_EncryptFinal_ex", "EVP_CIPHER_CTX_ctrl"):
    getattr(crypto, f).restype = ci
crypto.EVP_EncryptInit_ex.argtypes = [vp, vp, vp, cp, cp]
crypto.EVP_EncryptUpdate.argtypes = [vp, cp, ctypes.POINTER(ci), cp, ci]
crypto.EVP_EncryptFinal_ex.argtypes = [vp, cp, ctypes.POINTER(ci)]
crypto.EVP_CIPHER_CTX_ctrl.argtypes = [vp, ci, ci, vp]
crypto.EVP_CIPHER_CTX_free.argtypes = [vp]
EVP_CTRL_AEAD_SET_IVLEN, EVP_CTRL_AEAD_GET_TAG = 0x9, 0x10


def aead_encrypt(key: bytes, nonce: bytes, aad: bytes, pt: bytes):
    ctx = crypto.EVP_CIPHER_CTX_new()
    assert crypto.EVP_EncryptInit_ex(ctx, crypto.EVP_chacha20_poly1305(), None, None, None) == 1
    assert crypto.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, 12, None) == 1
    assert crypto.EVP_EncryptInit_ex(ctx, None, None, key, nonce) == 1
    n = ci(0)
    if aad:
        assert crypto.EVP_EncryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad)) == 1
    out = ctypes.create_string_buffer(len(pt) + 16)
    if pt:
        assert crypto.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), pt, len(pt)) == 1
        assert n.value == len(pt)
    assert crypto.EVP_EncryptFinal_ex(ctx, ctypes.cast(ctypes.byref(out, len(pt)), cp), ctypes.byref(n)) == 1
    tag = ctypes.create_string_buffer(16)
    assert crypto.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, ctypes.cast(tag, vp)) == 1
    crypto.EVP_CIPHER_CTX_free(ctx)
    return out.raw[: len(pt)], tag.raw


def chacha20_keystream(key: bytes, counter: int, nonce: bytes, n: int) -> bytes:
    ctx = crypto.EVP_CIPHER_CTX_new()
    iv = counter.to_bytes(4, "little") + nonce  # OpenSSL's 16-B chacha20 IV: counter || nonce
    assert crypto.EVP_EncryptInit_ex(ctx, crypto.EVP_chacha20(), None, key, iv) == 1
    out = ctypes.create_string_buffer(n)
    m = ci(0)
    assert crypto.EVP_EncryptUpdate(ctx, out, ctypes.byref(m), bytes(n), n) == 1
    crypto.EVP_CIPHER_CTX_free(ctx)
    return out.raw


def h(s: str) -> bytes:
    return bytes.fromhex(s.replace(" ", "").replace(":", ""))


RFC = {
    # RFC 8439 §2.3.2: block function, key 00..1f, counter 1
    "chacha20_block_2_3_2": {
        "key": bytes(range(32)).hex(), "counter": 1, "nonce": h("000000090000004a00000000").hex(),
        "keystream": h("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
                       "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e").hex()},
    # RFC 8439 §2.8.2: AEAD
    "aead_2_8_2": {
        "key": bytes(range(0x80, 0xa0)).hex(), "nonce": h("070000004041424344454647").hex(),
        "aad": h("50515253c0c1c2c3c4c5c6c7").hex(),
        "pt": (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for the future, "
               b"sunscreen would be it.").hex(),
        "tag": h("1ae10b594f09e26a7e902ecbd0600691").hex()},
}


def main():
    rfc = RFC["chacha20_block_2_3_2"]
    ks = chacha20_keystream(bytes.fromhex(rfc["key"]), rfc["counter"], bytes.fromhex(rfc["nonce"]), 64)
    assert ks.hex() == rfc["keystream"], "RFC 8439 §2.3.2 disagrees with OpenSSL"
    a = RFC["aead_2_8_2"]
    ct, tag = aead_encrypt(*(bytes.fromhex(a[k]) for k in ("key", "nonce", "aad", "pt")))
    assert tag.hex() == a["tag"], "RFC 8439 §2.8.2 tag disagrees with OpenSSL"
    a["ct"] = ct.hex()
    rng = random.Random(0x5EED00F4)
    cases = []
    lens = list(range(0, 70)) + [127, 128, 129, 255, 256, 257, 1023, 1024, 1025, 1440, 1460, 1472, 1500, 2047, 2048,
                                  2049, 4095, 4096, 4097, 9000]
    for n in lens:
        key = bytes(rng.getrandbits(8) for _ in range(32))
        nonce = bytes(rng.getrandbits(8) for _ in range(12))
        aad = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 0, 1, 12, 16, 33])))
        pt = bytes(rng.getrandbits(8) for _ in range(n))
        ct, tag = aead_encrypt(key, nonce, aad, pt)
        cases.append({"key": key.hex(), "nonce": nonce.hex(), "aad": aad.hex(), "pt": pt.hex(), "ct": ct.hex(),
                      "tag": tag.hex()})
    # WireGuard data messages: nonce = 4 zero bytes || le64(counter), no AAD,
    # plaintext zero-padded to 16 (proto/proto.cpp:557-583)
    wg = []
    for n in (0, 1, 15, 16, 17, 40, 64, 100, 1280, 1420, 1440, 1460, 1500):
        key = bytes(rng.getrandbits(8) for _ in range(32))
        counter = rng.choice([0, 1, 2, 0x1234, (1 << 32) + 7, (1 << 64) - (1 << 13) - 1])
        pt = bytes(rng.getrandbits(8) for _ in range(n))
        padded = pt + bytes(-n % 16)
        ct, tag = aead_encrypt(key, bytes(4) + counter.to_bytes(8, "little"), b"", padded)
        wg.append({"key": key.hex(), "counter": counter, "pt": pt.hex(), "ct": ct.hex(), "tag": tag.hex()})
    out = {"source": "OpenSSL " + ctypes.c_char_p(crypto.OpenSSL_version(0)).value.decode()
           if hasattr(crypto, "OpenSSL_version") else "OpenSSL libcrypto.so.3",
           "generator": "tests/golden/aead/gen_aead_golden.py", "rfc8439": RFC, "aead": cases, "wg": wg}
    (HERE / "aead_golden.json").write_text(json.dumps(out, indent=0) + "\n")
    print(f"{len(cases)} AEAD + {len(wg)} WireGuard vectors; RFC 8439 §2.3.2 and §2.8.2 confirmed by OpenSSL")


if __name__ == "__main__":
    crypto.OpenSSL_version.restype = ctypes.c_char_p
    crypto.OpenSSL_version.argtypes = [ci]
    main()
