"""PPM I/O for the path's output.

The reference prints P3 text, one "r g b" line per pixel (src/camera.h:35,
src/color.h:32-34).  Its committed image.ppm went through Windows PowerShell: UTF-16LE
with a BOM and CRLF line ends.  read_ppm() accepts that form, plain P3 and binary P6;
write_p3() is byte-identical to the reference's stdout; write_p6() is the compact binary
form of the same 8-bit values.
"""
from __future__ import annotations

import numpy as np


def normalize_text(raw: bytes) -> bytes:
    """UTF-16 (BOM) / CRLF -> the LF ASCII the reference binary prints."""
    if raw[:2] in (b"\xff\xfe", b"\xfe\xff"):
        raw = raw.decode("utf-16").encode("ascii")
    return raw.replace(b"\r\n", b"\n")


def read_ppm(data: bytes) -> np.ndarray:
    """-> int32 [H, W, 3]."""
    if data[:2] == b"P6":
        parts = data.split(maxsplit=4)
        w, h, maxval = int(parts[1]), int(parts[2]), int(parts[3])
        if maxval != 255:
            raise ValueError("only maxval 255")
        body = parts[4]
        return np.frombuffer(body[: w * h * 3], dtype=np.uint8).reshape(h, w, 3).astype(np.int32)
    text = normalize_text(data).decode("ascii")
    tok = text.split()
    if tok[0] != "P3":
        raise ValueError("not a PPM")
    w, h, maxval = int(tok[1]), int(tok[2]), int(tok[3])
    vals = np.array(tok[4:4 + w * h * 3], dtype=np.int64)
    if len(vals) != w * h * 3:
        raise ValueError("truncated PPM")
    return vals.astype(np.int32).reshape(h, w, 3)


def p3_bytes(rgb: np.ndarray) -> bytes:
    h, w, _ = rgb.shape
    head = f"P3\n{w} {h}\n255\n"
    return (head + "".join(f"{r} {g} {b}\n" for r, g, b in rgb.reshape(-1, 3).tolist())).encode("ascii")


def p6_bytes(rgb: np.ndarray) -> bytes:
    """Binary P6.  Values outside 0..255 (the INT_MIN a NaN sum prints) cannot be
    represented and raise."""
    if rgb.min() < 0 or rgb.max() > 255:
        raise ValueError("P6 holds 0..255 only (NaN pixels print INT_MIN in P3)")
    h, w, _ = rgb.shape
    return f"P6\n{w} {h}\n255\n".encode() + rgb.astype(np.uint8).tobytes()


def write_p3(path, rgb: np.ndarray) -> None:
    with open(path, "wb") as f:
        f.write(p3_bytes(rgb))


def write_p6(path, rgb: np.ndarray) -> None:
    with open(path, "wb") as f:
        f.write(p6_bytes(rgb))
