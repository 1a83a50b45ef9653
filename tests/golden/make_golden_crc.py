"""Generate tests/golden/crc_cases.json from the REFERENCE CRC-32 (7zCrc.c).

Run in the build container only (needs oracle/_ref/libref.so (container library) from
`make -f oracle/Makefile.ref`, which compiles 7zCrc.c / 7zCrcOpt.c /
CpuArch.c in place):

    python tests/golden/make_golden_crc.py

Each case names its input (explicit hex, or the synthetic generator
lzma-sdk-zliblike_amd/csrc/synth.c: kind, seed, length, then `skip` leading
bytes dropped so the range starts at every alignment) and records the
reference's CrcCalc(data) and CrcUpdate(0x12345678, data).
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import native  # noqa: E402

UPDATE_SEED = 0x12345678


def case_bytes(c):
    if "hex" in c:
        return bytes.fromhex(c["hex"])
    return native.gen(c["gen"], c["seed"], c["n"] + c["skip"])[c["skip"]:]


def main():
    lib = native.ref_cont()
    lib.CrcGenerateTable.restype = None
    lib.CrcGenerateTable()
    upd, calc = native.crc_funcs(lib, "CrcUpdate", "CrcCalc")
    cases = [{"hex": ""}, {"hex": "61"}, {"hex": b"123456789".hex()},
             {"hex": "00" * 32}, {"hex": "ff" * 33}]
    lengths = [1, 3, 4, 5, 15, 16, 17, 31, 63, 64, 65, 100, 2047, 2048, 2049, 4095, 4096,
               4097, 6143, 6144, 6145, 65536, 65537, 200003]
    k = 0
    for n in lengths:
        for gen in ("text", "random", "runs"):
            cases.append({"gen": gen, "seed": 700 + k, "n": n, "skip": k % 17})
            k += 1
    for c in cases:
        d = case_bytes(c)
        c["crc_calc"] = calc(d, len(d))
        c["crc_update"] = upd(UPDATE_SEED, d, len(d))
    with open(os.path.join(HERE, "crc_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_crc.py",
                   "reference": "LZMA SDK 9.20 7zCrc.c CrcCalc / CrcUpdate (oracle/Makefile.ref)",
                   "update_seed": UPDATE_SEED, "cases": cases}, f, indent=0)
    print(f"{len(cases)} CRC cases")


if __name__ == "__main__":
    main()
