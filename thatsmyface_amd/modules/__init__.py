"""Package-path compatible shim: ``from thatsmyface_amd.modules import watermarking``
mirrors the reference's ``from modules import watermarking``."""
