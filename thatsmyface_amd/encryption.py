"""Drop-in for the reference's modules/encryption.py (encrypt_watermark :8-40,
decrypt_watermark :43-68) on libtmfwm.so's AES-CBC (include/tmfwm.h tmfwm_aes_cbc_*), so the
pages work without pycryptodome (not in this image).  Same wire format: a random 16-byte IV
followed by AES-CBC of the PKCS#7-padded data; the key is 16, 24 or 32 bytes (the app passes
the 32-byte key of its fuzzy extractor).  decrypt_watermark returns None on any failure
(wrong key length, bad padding, truncated data), printing the error as the reference does.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Union

from . import _lib

BLOCK = 16


def _cbc(fn, key: bytes, iv: bytes, data: bytes) -> bytes:
    key, iv, data = bytes(key), bytes(iv), bytes(data)
    if len(key) not in (16, 24, 32):
        raise ValueError(f"Incorrect AES key length ({len(key)} bytes)")
    if len(iv) != BLOCK:
        raise ValueError("Incorrect IV length (it must be 16 bytes long)")
    if len(data) % BLOCK:
        raise ValueError("Data must be padded to 16 byte boundary in CBC mode")
    out = ctypes.create_string_buffer(max(len(data), 1))
    _lib.check(fn(key, len(key), iv, data, len(data), out), "aes_cbc")
    return out.raw[: len(data)]


def aes_cbc_encrypt(key: bytes, iv: bytes, data: bytes) -> bytes:
    return _cbc(_lib.load().tmfwm_aes_cbc_encrypt, key, iv, data)


def aes_cbc_decrypt(key: bytes, iv: bytes, data: bytes) -> bytes:
    return _cbc(_lib.load().tmfwm_aes_cbc_decrypt, key, iv, data)


def pad(data: bytes, block_size: int = BLOCK) -> bytes:
    """PKCS#7 (Crypto.Util.Padding.pad)."""
    n = block_size - len(data) % block_size
    return bytes(data) + bytes([n]) * n


def unpad(padded: bytes, block_size: int = BLOCK) -> bytes:
    """PKCS#7 (Crypto.Util.Padding.unpad), with its checks."""
    if len(padded) == 0:
        raise ValueError("Zero-length input cannot be unpadded")
    if len(padded) % block_size:
        raise ValueError("Input data is not padded")
    n = padded[-1]
    if n < 1 or n > min(block_size, len(padded)):
        raise ValueError("Padding is incorrect.")
    if padded[-n:] != bytes([n]) * n:
        raise ValueError("PKCS#7 padding is incorrect.")
    return padded[:-n]


def encrypt_watermark(watermark_data: Union[str, bytes], key: bytes) -> bytes:
    data = watermark_data.encode("utf-8") if isinstance(watermark_data, str) else watermark_data
    iv = os.urandom(BLOCK)  # get_random_bytes(16)
    return iv + aes_cbc_encrypt(key, iv, pad(data, BLOCK))


def decrypt_watermark(encrypted_data: bytes, key: bytes) -> Optional[bytes]:
    try:
        iv, ciphertext = encrypted_data[:BLOCK], encrypted_data[BLOCK:]
        return unpad(aes_cbc_decrypt(key, iv, ciphertext), BLOCK)
    except Exception as e:
        print(f"Decryption error: {str(e)}")
        return None
