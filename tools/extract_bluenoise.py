"""Extract the blue-noise sampler tables of RenderCore_OptixPrime_B into a binary asset.

The reference compiles three 8-bit tables (Heitz et al., "A Low-Discrepancy Sampler that
Distributes Monte Carlo Errors as a Blue Noise in Screen Space", tables from
https://eheitzresearch.wordpress.com/762-2) into core_settings.h as uint64 literals
(lib/RenderCore_OptixPrime_B/core_settings.h:167, 297, 555) and expands them to one uint32 per
byte at start-up (rendercore.cpp:125-134):
    data32[i]             = sob256_64 bytes, i <  65536
    data32[65536 + i]     = scr256_64 bytes, i < 131072
    data32[3*65536 + i]   = rnk256_64 bytes, i < 131072
This script (run once, in the container that has /root/reference) writes those 327680 bytes to
lighthouse2_amd/data/bluenoise.bin; the GPU box only ever sees the .bin.
"""
import pathlib
import re
import sys

import numpy as np

REF = pathlib.Path("/root/reference/lib/RenderCore_OptixPrime_B/core_settings.h")
OUT = pathlib.Path(__file__).resolve().parents[1] / "lighthouse2_amd" / "data" / "bluenoise.bin"


def table(text: str, name: str, count: int) -> np.ndarray:
    m = re.search(r"const uint64_t " + name + r"\[(\d+)\]\s*=\s*\{(.*?)\};", text, re.S)
    if not m or int(m.group(1)) != count:
        raise SystemExit(f"table {name} not found")
    vals = [int(v, 16) for v in re.findall(r"0x[0-9a-fA-F]+", m.group(2))]
    assert len(vals) == count, (name, len(vals))
    return np.array(vals, dtype="<u8").view(np.uint8)  # little-endian byte order (x86 / GPU)


def main() -> None:
    text = REF.read_text()
    sob = table(text, "sob256_64", 8192)     # 65536 bytes
    scr = table(text, "scr256_64", 16384)    # 131072 bytes
    rnk = table(text, "rnk256_64", 16384)    # 131072 bytes
    out = np.zeros(65536 * 5, dtype=np.uint8)
    out[:65536] = sob
    out[65536:65536 + 131072] = scr
    out[3 * 65536:3 * 65536 + 131072] = rnk
    OUT.parent.mkdir(parents=True, exist_ok=True)
    out.tofile(OUT)
    print(f"wrote {OUT} ({out.nbytes} bytes)", file=sys.stderr)


if __name__ == "__main__":
    main()
