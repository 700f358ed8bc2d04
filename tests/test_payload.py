"""The watermark's payload codec: AES-CBC and the QR codec of
libtmfwm.so (host C++, include/tmfwm.h tmfwm_aes_* / tmfwm_qr_*) behind the drop-ins
thatsmyface_amd.encryption / thatsmyface_amd.qrcode_generator.

pycryptodome, python-qrcode and pyzbar are not in this image, so parity is pinned by the
published standards' known answers (FIPS-197 appendix C, SP 800-38A F.2 for AES; ISO/IEC
18004's BCH words and Reed-Solomon code for QR) and by round trips through the watermark
path itself (the reference's own use: encrypt -> QR -> embed | extract -> decode -> decrypt,
embed_watermark_page.py:480-531, extract_watermark_page.py:293-364).  QR byte-equality with
python-qrcode's output is "parity unpinned".
"""
import base64
import io

import numpy as np
import pytest
from PIL import Image

from oracle import oracle as O
from thatsmyface_amd import _lib
from thatsmyface_amd import encryption as E
from thatsmyface_amd import qrcode_generator as Q

PT = bytes.fromhex("00112233445566778899aabbccddeeff")


@pytest.mark.parametrize("key,ct", [
    ("000102030405060708090a0b0c0d0e0f", "69c4e0d86a7b0430d8cdb78070b4c55a"),  # FIPS-197 C.1
    ("000102030405060708090a0b0c0d0e0f1011121314151617", "dda97ca4864cdfe06eaf70a0ec0d7191"),  # C.2
    ("000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f", "8ea2b7ca516745bfeafc49904b496089"),  # C.3
])
def test_aes_fips197(key, ct):
    k = bytes.fromhex(key)
    assert E.aes_cbc_encrypt(k, bytes(16), PT).hex() == ct  # one CBC block with a zero IV = the cipher
    assert E.aes_cbc_decrypt(k, bytes(16), bytes.fromhex(ct)) == PT


def test_aes_cbc_sp800_38a():
    """SP 800-38A F.2.5 / F.2.6 (CBC-AES256), four blocks, and in-place decryption."""
    k = bytes.fromhex("603deb1015ca71be2b73aef0857d77811f352c073b6108d72d9810a30914dff4")
    iv = bytes.fromhex("000102030405060708090a0b0c0d0e0f")
    p = bytes.fromhex("6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e51"
                      "30c81c46a35ce411e5fbc1191a0a52eff69f2445df4f9b17ad2b417be66c3710")
    c = bytes.fromhex("f58c4c04d6e5f1ba779eabfb5f7bfbd69cfc4e967edb808d679f777bc6702c7d"
                      "39f23369a9d9bacfa530e26304231461b2eb05e2c39be9fcda6c19078c6a9d1b")
    assert E.aes_cbc_encrypt(k, iv, p) == c
    assert E.aes_cbc_decrypt(k, iv, c) == p
    L = _lib.load()
    buf = bytearray(c)
    arr = (np.frombuffer(buf, np.uint8))
    _lib.check(L.tmfwm_aes_cbc_decrypt(k, 32, iv, arr.ctypes.data, len(buf), arr.ctypes.data), "in place")
    assert bytes(buf) == p


def test_encrypt_decrypt_watermark_contract():
    """encryption.py:8-68: IV || CBC(PKCS#7(data)); fresh IV per call; None on every failure."""
    key = bytes(range(32))
    for data in ("", "hello", "x" * 16, "ünïcödé ✓", b"\x00\xff" * 40):
        a, b = E.encrypt_watermark(data, key), E.encrypt_watermark(data, key)
        raw = data.encode() if isinstance(data, str) else data
        assert len(a) == 16 + (len(raw) // 16 + 1) * 16 and a[:16] != b[:16]
        assert E.decrypt_watermark(a, key) == raw
        assert E.unpad(E.aes_cbc_decrypt(key, a[:16], a[16:])) == raw
    enc = E.encrypt_watermark("secret", key)
    assert E.decrypt_watermark(enc, bytes(32)) in (None, b"secret") and E.decrypt_watermark(enc, bytes(32)) != b"secret"
    assert E.decrypt_watermark(enc, key[:20]) is None  # bad key length
    assert E.decrypt_watermark(enc[:-1], key) is None  # not a block multiple
    assert E.decrypt_watermark(enc[:16], key) is None  # zero-length ciphertext
    assert E.decrypt_watermark(b"short", key) is None  # short IV
    for key_len in (16, 24):
        k = bytes(range(key_len))
        assert E.decrypt_watermark(E.encrypt_watermark("aes-%d" % (8 * key_len), k), k) == b"aes-%d" % (8 * key_len)


def _symbol_image(m, scale=4):
    g = np.where(np.pad(m, 4), 0, 255).astype(np.uint8)
    return np.kron(g, np.ones((scale, scale), np.uint8))


def test_qr_format_and_version_words():
    """ISO 18004 BCH words: format (level M, mask 0 / level H, mask 7 ...) and version 7."""
    rng = np.random.default_rng(1)
    for lvl, data in ((3, b"H level"), (0, b"L level"), (1, b"M"), (2, b"Q" * 9)):
        m = Q.qr_matrix(data, lvl, 1)
        n = m.shape[0]
        # both copies of the 15 format bits agree (col 8 / row 8 paths)
        col = [m[i if i < 6 else (i + 1 if i < 8 else n - 15 + i), 8] for i in range(15)]
        row = [m[8, n - i - 1 if i < 8 else (15 - i if i < 9 else 14 - i)] for i in range(15)]
        assert col == row
        assert m[n - 8, 8]  # dark module
        word = sum(int(b) << i for i, b in enumerate(col)) ^ 0x5412
        assert (word >> 13) == {0: 1, 1: 0, 2: 3, 3: 2}[lvl]  # level bits in the top two data bits
    m = Q.qr_matrix(bytes(rng.integers(0, 256, 120).astype(np.uint8)), 0, 7)
    assert m.shape[0] == 45  # version 7 requested as the minimum
    bits = sum(int(m[i // 3, 45 - 11 + i % 3]) << i for i in range(18))
    assert bits == 0x07C94  # the standard's version-7 information word
    assert bits == sum(int(m[45 - 11 + i % 3, i // 3]) << i for i in range(18))


@pytest.mark.parametrize("lvl", [0, 1, 2, 3])
def test_qr_round_trip_all_versions(lvl):
    rng = np.random.default_rng(lvl)
    seen = set()
    for n in range(1, 272, 7):
        data = bytes(rng.integers(0, 256, n).astype(np.uint8))
        try:
            m = Q.qr_matrix(data, lvl, 1)
        except NotImplementedError:
            break  # beyond version 10
        seen.add(m.shape[0])
        assert Q.decode_image(_symbol_image(m, 3)) == data
    assert len(seen) == 10  # versions 1..10 all exercised


def test_qr_segments_numeric_alphanumeric():
    """python-qrcode's segmentation: >= 20-digit runs numeric, >= 20-char alphanumeric runs."""
    for text in (b"12345678901234567890123", b"HELLO WORLD THIS IS ALNUM 123", b"abc" + b"0" * 25 + b"xyz",
                 b"ABCDEFGHIJKLMNOPQRSTUVWXYZ/abc+123", b"1234", b"ABC DEF", b"0" * 100):
        m = Q.qr_matrix(text, 3, 1)
        assert Q.decode_image(_symbol_image(m)) == text
    # numeric mode is denser: 100 digits fit version 5 at H (byte mode would need version 6)
    assert Q.qr_matrix(b"0" * 100, 3, 1).shape[0] == 37


def test_qr_error_correction():
    """Reed-Solomon: flipped modules up to what level H corrects are repaired."""
    rng = np.random.default_rng(3)
    data = base64.b64encode(bytes(range(48)))
    m = Q.qr_matrix(data, 3, 1)
    n = m.shape[0]
    fn = np.zeros_like(m)  # keep finder / timing / format areas intact
    fn[:9, :9] = fn[:9, n - 8:] = fn[n - 8:, :9] = True
    fn[6, :] = fn[:, 6] = True
    cand = np.argwhere(~fn)
    for k in (5, 20, 40):
        bad = m.copy()
        for r, c in cand[rng.choice(len(cand), k, replace=False)]:
            bad[r, c] = ~bad[r, c]
        assert Q.decode_image(_symbol_image(bad)) == data, k
    assert Q.decode_image(np.full((50, 50), 255, np.uint8)) is None


def test_text_to_qrcode_contract():
    """qrcode_generator.py:10-44: base64 of bytes, H level, box 10, border 4, mode "1", 300 x 300."""
    enc = E.encrypt_watermark("payload", bytes(32))
    img = Q.text_to_qrcode(enc)
    assert img.mode == "1" and img.size == (300, 300)
    m = Q.qr_matrix(base64.b64encode(enc), 3, 1)
    full = Q.render(m)
    assert full.size == ((m.shape[0] + 8) * 10,) * 2
    assert np.array_equal(np.asarray(img), np.asarray(full.resize((300, 300), Image.NEAREST)))
    assert Q.qrcode_to_text(img) == enc
    assert Q.qrcode_to_text(Q.text_to_qrcode("plain text, not base64!")) == "plain text, not base64!"
    assert Q.qrcode_to_text(Image.new("L", (40, 40), 255)) is None


@pytest.mark.parametrize("b,alpha", [(8, 0.1), (8, 0.5), (16, 0.1), (12, 0.2)])
def test_app_round_trip_through_the_watermark(b, alpha):
    """The app's loop on the oracle (CPU stand-in for the GPU kernels): encrypt -> QR -> PNG ->
    resize_watermark(preserve_ratio) -> embed | extract -> qrcode_to_text -> decrypt."""
    from lapack_path import photo_cover

    key = bytes(range(100, 132))
    enc = E.encrypt_watermark("ThatsMyFace", key)
    buf = io.BytesIO()
    Q.text_to_qrcode(enc).save(buf, format="PNG")
    wm = np.asarray(Image.open(io.BytesIO(buf.getvalue())).convert("L"))
    H, W = 1088, 1920
    cov = photo_cover(H, W, 9)
    tile = O.prepare_tile(wm, H // b, W // b, True)
    ext = O.extract_frame(O.embed_frame(cov, tile, b, alpha), cov, b, alpha)
    got = Q.qrcode_to_text(Image.fromarray(ext))
    assert got == enc
    assert E.decrypt_watermark(got, key) == b"ThatsMyFace"
    assert Q.decode_tiles(np.stack([ext, ext])) == [base64.b64encode(enc)] * 2
