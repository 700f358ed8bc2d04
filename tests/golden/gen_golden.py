#!/usr/bin/env python3
"""Generate the golden fixtures by running the REFERENCE itself.

Container-only: imports /root/reference/modules/watermarking.py read-only with a
``streamlit`` stub (streamlit is not installed; the module imports it at top
level, watermarking.py:5, but only uses it inside get_watermark_settings
:14-15, which is bypassed by passing ``custom_settings``).  Nothing from the
reference is copied: the fixtures are inputs and the reference's outputs.

Outputs (tests/golden/):
  cases.npz        end-to-end cases: cover, watermark, settings -> resized tile,
                   embed_watermark RGB, extract_watermark L   (watermarking.py:135, :224)
  stages.npz       per-stage intermediates for one cover: Y plane (:166-169),
                   DCT blocks (:192), LAPACK S (:195), reconstructed M (:198-201),
                   IDCT blocks (:204) and the final RGB (:216)
  meta.json        library versions, KAT hashes re-derived here,
                   per-case sha256 of every expected output

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py            (cases.npz, stages.npz, meta.json)
      PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py --blocks   (cases_blocks.npz, meta_blocks.json)
      PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py --alpha    (cases_alpha.npz, meta_alpha.json)
      PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py --helpers  (helpers.npz, meta_helpers.json)
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    st = types.ModuleType("streamlit")
    st.session_state = {}
    sys.modules["streamlit"] = st
    sys.path.insert(0, REF)
    import modules.watermarking as W  # noqa: E402

    return W


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ---------------------------------------------------------------- covers
def cover(kind: str, H: int, W: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    y, x = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    if kind == "noise":
        return rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    if kind == "pattern":  # KAT-A/B cover
        c = np.arange(3)[None, None, :]
        return ((7 * x[..., None] + 13 * y[..., None] + 29 * c) % 256).astype(np.uint8)
    if kind == "smooth":
        r = (x * 255 // max(W - 1, 1)).astype(np.uint8)
        g = (y * 255 // max(H - 1, 1)).astype(np.uint8)
        b = ((x + y) * 127 // max(H + W - 2, 1)).astype(np.uint8)
        return np.stack([r, g, b], -1)
    if kind == "flat":
        out = np.empty((H, W, 3), np.uint8)
        out[...] = (90, 140, 200)
        return out
    if kind == "black":
        return np.zeros((H, W, 3), np.uint8)
    if kind == "qr":  # binary 0/255 modules of 4 px, like a QR code cover
        m = rng.integers(0, 2, ((H + 3) // 4, (W + 3) // 4), dtype=np.uint8) * 255
        m = np.kron(m, np.ones((4, 4), np.uint8))[:H, :W]
        return np.stack([m] * 3, -1)
    if kind == "blocky":
        m = rng.integers(0, 256, ((H + 7) // 8, (W + 7) // 8, 3), dtype=np.uint8)
        return np.kron(m, np.ones((8, 8, 1), np.uint8))[:H, :W]
    if kind == "diagonal":
        v = (((x + y) // 3) % 2 * 200 + 30).astype(np.uint8)
        return np.stack([v, v // 2, 255 - v], -1)
    if kind == "xor":  # KAT-C luma pattern
        v = ((y ^ x) & 255).astype(np.uint8)
        return v
    raise ValueError(kind)


def wmark(kind: str, h: int, w: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    i, j = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    if kind == "noise":
        return rng.integers(0, 256, (h, w), dtype=np.uint8)
    if kind == "pattern":
        return ((37 * i + 11 * j) % 256).astype(np.uint8)
    if kind == "mul":
        return ((i * j) & 255).astype(np.uint8)
    if kind == "qr":
        return (rng.integers(0, 2, (h, w), dtype=np.uint8) * 255).astype(np.uint8)
    raise ValueError(kind)


# (name, cover kind, H, W, cover mode, wm kind, wm h, wm w, wm as bytes, block, alpha, preserve_ratio)
CASES = [
    ("kat_a", "pattern", 64, 64, "RGB", "pattern", 8, 8, False, 8, 0.1, False),
    ("kat_b", "pattern", 64, 64, "RGB", "pattern", 4, 4, False, 16, 0.2, False),
    ("kat_c", "xor", 512, 512, "L", "mul", 64, 64, False, 8, 0.1, False),
    ("noise_128x96_pr", "noise", 128, 96, "RGB", "noise", 20, 30, True, 8, 0.1, True),
    ("smooth_250x333_pr", "smooth", 250, 333, "RGB", "qr", 33, 33, True, 8, 0.05, True),
    ("flat_64x80", "flat", 64, 80, "RGB", "noise", 8, 10, False, 8, 0.15, False),
    ("black_96", "black", 96, 96, "RGB", "qr", 29, 29, True, 8, 0.1, True),
    ("qr_cover_160", "qr", 160, 160, "RGB", "qr", 21, 21, True, 8, 0.1, True),
    ("blocky_128_b16", "blocky", 128, 128, "RGB", "noise", 8, 8, False, 16, 0.01, False),
    ("diag_100x140_b4", "diagonal", 100, 140, "RGB", "pattern", 25, 35, False, 4, 0.2, False),
    ("rgba_72x64", "noise", 72, 64, "RGBA", "noise", 9, 8, False, 8, 0.1, False),
    ("lmode_64", "noise", 64, 64, "L", "noise", 8, 8, True, 8, 0.1, False),
    ("noise_136x200_b16", "noise", 136, 200, "RGB", "noise", 40, 40, False, 16, 0.1, False),
    ("noise_256_a", "noise", 256, 256, "RGB", "noise", 32, 32, False, 8, 0.1, False),
    ("noise_256_b", "noise", 256, 256, "RGB", "qr", 45, 45, True, 8, 0.2, True),
    ("smooth_256_b8", "smooth", 256, 256, "RGB", "noise", 32, 32, False, 8, 0.1, False),
    ("qr_cover_256_b16", "qr", 256, 256, "RGB", "qr", 16, 16, False, 16, 0.15, False),
] + [
    (f"sweep_b16_a{a}", "noise", 128, 128, "RGB", "noise", 8, 8, False, 16, a, False)
    for a in (0.01, 0.05, 0.1, 0.15, 0.2)
] + [
    (f"sweep_b8_a{a}", "smooth", 96, 128, "RGB", "noise", 12, 16, False, 8, a, False)
    for a in (0.01, 0.05, 0.15, 0.2)
]


# UI slider block sizes beyond 4/8/16 (embed_watermark_page.py:324-331): pocketfft
# radix 3 (6, 12), 5 (10) and generic 7 (14).  Written to cases_blocks.npz /
# meta_blocks.json by `gen_golden.py --blocks`, so the fixtures above stay as they are.
BLOCK_CASES = [
    ("noise_120x180_b6", "noise", 120, 180, "RGB", "noise", 20, 30, False, 6, 0.1, False),
    ("diag_100x97_b6", "diagonal", 100, 97, "RGB", "pattern", 16, 16, False, 6, 0.15, False),
    ("lmode_xor_96_b6", "xor", 96, 96, "L", "mul", 16, 16, False, 6, 0.1, False),
    ("noise_125x173_b10_pr", "noise", 125, 173, "RGB", "qr", 21, 21, True, 10, 0.1, True),
    ("smooth_150x200_b10", "smooth", 150, 200, "RGB", "noise", 15, 20, False, 10, 0.05, False),
    ("noise_144x156_b12", "noise", 144, 156, "RGB", "noise", 12, 13, False, 12, 0.2, False),
    ("blocky_120x130_b12", "blocky", 120, 130, "RGB", "noise", 10, 10, False, 12, 0.1, False),
    ("noise_140x154_b14", "noise", 140, 154, "RGB", "noise", 10, 11, False, 14, 0.1, False),
    ("rgba_112x126_b14", "noise", 112, 126, "RGBA", "pattern", 8, 9, False, 14, 0.15, False),
    ("flat_84x84_b14", "flat", 84, 84, "RGB", "qr", 6, 6, False, 14, 0.1, False),
]


# The app's alpha slider goes to 1.0 (embed_watermark_page.py:343-350); the configs stop
# at 0.2.  Written to cases_alpha.npz / meta_alpha.json by `gen_golden.py --alpha`.
# Larger alpha pushes S[0] further from the cover's spectrum: more clipping in the inverse
# colour and larger extract values (no saturation at 255 until alpha * w / 255 >= ...).
ALPHA_CASES = [
    (f"{kind}_{H}x{W}_b{b}_a{a}", kind, H, W, "RGB", wk, H // b, W // b, False, b, a, False)
    for (kind, H, W, wk) in (("noise", 96, 128, "noise"), ("smooth", 112, 96, "qr"), ("qr", 128, 128, "qr"))
    for b in (8, 16)
    for a in (0.3, 0.5, 0.75, 1.0)
] + [
    ("noise_120x180_b6_a1.0", "noise", 120, 180, "RGB", "noise", 20, 30, False, 6, 1.0, False),
    ("blocky_120x130_b12_a0.5", "blocky", 120, 130, "RGB", "noise", 10, 10, False, 12, 0.5, False),
    ("noise_150x200_b10_a0.5_pr", "noise", 150, 200, "RGB", "qr", 21, 21, True, 10, 0.5, True),
    ("diag_84x84_b14_a1.0", "diagonal", 84, 84, "RGB", "pattern", 6, 6, False, 14, 1.0, False),
    ("noise_100x140_b4_a0.5", "noise", 100, 140, "RGB", "noise", 25, 35, False, 4, 0.5, False),
]


def _mode_img(arr: np.ndarray, mode: str):
    from PIL import Image

    if mode == "L":
        return Image.fromarray(arr if arr.ndim == 2 else arr[..., 0], "L")
    if mode == "RGBA":
        a = np.full(arr.shape[:2] + (1,), 77, np.uint8)
        return Image.fromarray(np.concatenate([arr, a], -1), "RGBA")
    return Image.fromarray(arr, "RGB")


def run_cases(W, cases, seed_base: int, out: dict, meta: dict) -> None:
    """embed_watermark / extract_watermark of the reference on every case."""
    from PIL import Image

    for seed, (name, ck, H, Wd, cmode, wk, wh, ww, as_bytes, b, alpha, pr) in enumerate(cases):
        carr = cover(ck, H, Wd, seed_base + seed)
        cimg = _mode_img(carr, cmode)
        warr = wmark(wk, wh, ww, seed_base + 1000 + seed)
        wimg = Image.fromarray(warr, "L")
        if as_bytes:
            buf = io.BytesIO()
            wimg.save(buf, format="PNG")
            wdata = buf.getvalue()
        else:
            wdata = wimg
        settings = {"block_size": b, "alpha": alpha}
        emb = W.embed_watermark(cimg, wdata, pr, settings)
        ext = W.extract_watermark(emb, cimg, settings)
        tile = W.resize_watermark(wdata, H // b, Wd // b, pr)
        cin = np.asarray(cimg)
        e_arr, x_arr, t_arr = np.asarray(emb), np.asarray(ext), np.asarray(tile)
        out[f"{name}/cover"] = cin
        out[f"{name}/wm"] = warr
        out[f"{name}/tile"] = t_arr
        out[f"{name}/embed"] = e_arr
        out[f"{name}/extract"] = x_arr
        meta["cases"][name] = {
            "cover_kind": ck, "cover_mode": cimg.mode, "H": H, "W": Wd, "wm_kind": wk,
            "wm_as_png_bytes": as_bytes, "block": b, "alpha": alpha, "preserve_ratio": pr,
            "embed_mode": emb.mode, "extract_mode": ext.mode,
            "sha_embed": sha(e_arr), "sha_extract": sha(x_arr), "sha_tile": sha(t_arr),
        }
        print(name, cimg.mode, e_arr.shape, x_arr.shape, flush=True)


def main_blocks() -> None:
    """cases_blocks.npz + meta_blocks.json: block sizes 6, 10, 12, 14."""
    import PIL
    import scipy

    W = _import_reference()
    out: dict[str, np.ndarray] = {}
    meta: dict = {"generator": "tests/golden/gen_golden.py --blocks",
                  "reference": "/root/reference/modules/watermarking.py (embed_watermark :135, extract_watermark :224)",
                  "numpy": np.__version__, "scipy": scipy.__version__, "pillow": PIL.__version__, "cases": {}}
    run_cases(W, BLOCK_CASES, 3000, out, meta)
    np.savez_compressed(os.path.join(HERE, "cases_blocks.npz"), **out)
    with open(os.path.join(HERE, "meta_blocks.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote cases_blocks.npz, meta_blocks.json")


def main_alpha() -> None:
    """cases_alpha.npz + meta_alpha.json: the app's alpha slider range up to 1.0."""
    import PIL
    import scipy

    W = _import_reference()
    out: dict[str, np.ndarray] = {}
    meta: dict = {"generator": "tests/golden/gen_golden.py --alpha",
                  "reference": "/root/reference/modules/watermarking.py (embed_watermark :135, extract_watermark :224)",
                  "numpy": np.__version__, "scipy": scipy.__version__, "pillow": PIL.__version__, "cases": {}}
    run_cases(W, ALPHA_CASES, 5000, out, meta)
    np.savez_compressed(os.path.join(HERE, "cases_alpha.npz"), **out)
    with open(os.path.join(HERE, "meta_alpha.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote cases_alpha.npz, meta_alpha.json")


def main() -> None:
    from PIL import Image

    W = _import_reference()
    out: dict[str, np.ndarray] = {}
    meta: dict = {
        "generator": "tests/golden/gen_golden.py",
        "reference": "/root/reference/modules/watermarking.py (embed_watermark :135, extract_watermark :224)",
        "numpy": np.__version__,
        "cases": {},
    }
    import PIL
    import scipy

    meta["scipy"] = scipy.__version__
    meta["pillow"] = PIL.__version__
    run_cases(W, CASES, 1000, out, meta)

    # ---- per-stage intermediates on one noise cover (watermarking.py:166-216)
    carr = cover("noise", 64, 48, 77)
    warr = wmark("noise", 8, 6, 78)
    b, alpha = 8, 0.1
    ycc = W.rgb_to_ycbcr(Image.fromarray(carr))
    Y = ycc[:, :, 0].copy()
    nbh, nbw = 64 // b, 48 // b
    D, S, M, Yb = [], [], [], []
    wtile = np.asarray(W.resize_watermark(Image.fromarray(warr), nbh, nbw, False)) / 255.0
    Ymod = Y.copy()
    for i in range(nbh):
        for j in range(nbw):
            blk = Y[i * b:(i + 1) * b, j * b:(j + 1) * b]
            d = W.apply_dct_to_block(blk)
            u, s, vt = np.linalg.svd(d, full_matrices=True)
            s0 = s.copy()
            s[0] += alpha * wtile[i, j]
            m = np.dot(u, np.dot(np.diag(s), vt))
            y2 = W.apply_idct_to_block(m)
            D.append(d); S.append(s0); M.append(m); Yb.append(y2)
            Ymod[i * b:(i + 1) * b, j * b:(j + 1) * b] = y2
    ycc2 = ycc.copy()
    ycc2[:, :, 0] = Ymod
    rgb2 = W.ycbcr_to_rgb(ycc2)
    stages = {
        "cover": carr, "wm": warr, "ycc": ycc, "D": np.stack(D), "S": np.stack(S),
        "M": np.stack(M), "Yblocks": np.stack(Yb), "rgb_out": rgb2,
        "block": np.int32(b), "alpha": np.float64(alpha),
    }
    np.savez_compressed(os.path.join(HERE, "stages.npz"), **stages)

    # ---- KATs, re-derived with the reference here
    kats = {}
    idx = np.arange(1 << 12, dtype=np.uint32)
    # 2^24-colour tables: run the reference's per-pixel loops over all colours (~1 min)
    if os.environ.get("TMF_GOLDEN_TABLES", "1") == "1":
        allc = np.arange(1 << 24, dtype=np.uint32)
        rgb = np.stack([(allc >> 16) & 255, (allc >> 8) & 255, allc & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)
        tab = W.rgb_to_ycbcr(Image.fromarray(rgb))
        kats["colour_fwd_table_sha256"] = sha(tab)
        kats["colour_roundtrip_table_sha256"] = sha(W.ycbcr_to_rgb(tab))
        del tab, rgb
    del idx
    meta["kats"] = kats
    np.savez_compressed(os.path.join(HERE, "cases.npz"), **out)
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", os.listdir(HERE))


def helper_inputs() -> dict[str, np.ndarray]:
    """Non-uint8 inputs of the module-level colour helpers (watermarking.py:23, :53)."""
    rng = np.random.default_rng(2026)
    special = np.array([0.0, 255.0, 254.5, 0.5, -0.0, 1e-3, 1e6, 127.5, 256.0, -1.0, 3.0, 254.999],
                       np.float64).reshape(2, 2, 3)
    ycc = np.stack([rng.uniform(-0.3, 1.3, (24, 24)), rng.uniform(-0.3, 1.3, (24, 24)), rng.uniform(-0.3, 1.3, (24, 24))], -1)
    k = np.arange(256, dtype=np.float64)
    y = np.concatenate([(k - 1e-9) / 255, (k + 1e-9) / 255, np.nextafter(k / 255, -1), k / 255])
    edge = np.stack([y, np.full_like(y, 0.5), np.full_like(y, 0.5)], -1).reshape(32, 32, 3)
    return {
        "fwd_f32": rng.uniform(-30, 290, (24, 24, 3)).astype(np.float32),
        "fwd_f64": rng.uniform(-30, 290, (24, 24, 3)),
        "fwd_special_f64": special,
        "fwd_i32": rng.integers(-100, 400, (24, 24, 3), dtype=np.int32),
        "fwd_u16": rng.integers(0, 65536, (16, 16, 3), dtype=np.uint16),
        "fwd_rgba_f64": rng.uniform(0, 255, (8, 8, 4)),
        "inv_f64": ycc,
        "inv_f32": ycc.astype(np.float32),
        "inv_f16": ycc.astype(np.float16),
        # truncation edges: Y just below / above k / 255, neutral chroma
        "inv_edge_f64": edge,
        "inv_edge_f16": edge.astype(np.float16),
        "noise_u8": rng.integers(0, 256, (24, 24, 3), dtype=np.uint8),
    }


def main_helpers() -> None:
    """helpers.npz + meta_helpers.json: rgb_to_ycbcr on non-uint8 arrays and
    ycbcr_to_rgb on float16 / float32 / float64 arrays, outputs by the reference."""
    W = _import_reference()
    inp = helper_inputs()
    out: dict[str, np.ndarray] = {}
    for k, v in inp.items():
        out["in_" + k] = v
        if k.startswith("fwd_"):
            out["out_" + k] = W.rgb_to_ycbcr(v)
        elif k.startswith("inv_"):
            out["out_" + k] = W.ycbcr_to_rgb(v)
    ycc = W.rgb_to_ycbcr(inp["noise_u8"])
    for dt in ("f16", "f64"):
        a = ycc.astype(np.float16 if dt == "f16" else np.float64)
        out[f"in_inv_noise_{dt}"] = a
        out[f"out_inv_noise_{dt}"] = W.ycbcr_to_rgb(a)
    del out["in_noise_u8"]
    np.savez_compressed(os.path.join(HERE, "helpers.npz"), **out)
    meta = {"generator": "tests/golden/gen_golden.py --helpers",
            "reference": "/root/reference/modules/watermarking.py (rgb_to_ycbcr :23, ycbcr_to_rgb :53)",
            "numpy": np.__version__, "sha": {k: sha(v) for k, v in sorted(out.items())}}
    with open(os.path.join(HERE, "meta_helpers.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote helpers.npz:", sorted(out))


if __name__ == "__main__":
    if "--helpers" in sys.argv[1:]:
        main_helpers()
    elif "--blocks" in sys.argv[1:]:
        main_blocks()
    elif "--alpha" in sys.argv[1:]:
        main_alpha()
    else:
        main()
