"""Same module path as the reference's modules/encryption.py."""
from ..encryption import decrypt_watermark, encrypt_watermark  # noqa: F401
