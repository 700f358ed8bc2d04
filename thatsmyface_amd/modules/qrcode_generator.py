"""Same module path as the reference's modules/qrcode_generator.py."""
from ..qrcode_generator import qrcode_to_text, text_to_qrcode  # noqa: F401
