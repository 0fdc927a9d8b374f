"""Extract the reference's own known-answer vectors as data fixtures (tests/golden/).

Reads the Go test sources of the reference AS TEXT (nothing is compiled or
executed) and writes the embedded test DATA only:

  bitpack32_kats.json   127 vectors of bitpacking32_test.go (unpack8int32Tests)
  bitpack64_kats.json   317 vectors of bitpacking64_test.go (unpack8int64Tests)
  must_not_crash/*.bin  the adversarial file images embedded in the fuzz
                        regression tests (fuzz_test.go, deltabp_decoder_test.go,
                        type_dict_test.go, page_v1_test.go, chunk_reader_test.go,
                        type_bytearray_test.go, schema_test.go)

Run in the build container (the reference tree is not present on the GPU box):
    python tools/extract_reference_kats.py /root/reference
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def parse_int(tok):
    tok = tok.strip()
    return int(tok, 0)


def kats(path, bits):
    src = open(path).read()
    pat = re.compile(r"\{\s*(\d+)\s*,\s*\[\]byte\{([^}]*)\}\s*,\s*\[8\]int%d\{([^}]*)\}\s*,?\s*\}" % bits)
    out = []
    for m in pat.finditer(src):
        width = int(m.group(1))
        data = [parse_int(x) for x in m.group(2).split(",") if x.strip()]
        vals = [parse_int(x) for x in m.group(3).split(",") if x.strip()]
        assert len(vals) == 8
        out.append({"width": width, "data": data, "values": vals})
    return out


_ESC = {"a": 7, "b": 8, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11, "\\": 92, '"': 34, "'": 39}


def go_string(lit):
    """Decode one Go interpreted string literal body (between the quotes) to bytes."""
    out = bytearray()
    i = 0
    while i < len(lit):
        c = lit[i]
        if c != "\\":
            out += c.encode("utf-8")
            i += 1
            continue
        n = lit[i + 1]
        if n == "x":
            out.append(int(lit[i + 2:i + 4], 16))
            i += 4
        elif n == "u":
            out += chr(int(lit[i + 2:i + 6], 16)).encode("utf-8")
            i += 6
        elif n == "U":
            out += chr(int(lit[i + 2:i + 10], 16)).encode("utf-8")
            i += 10
        elif n in "01234567":
            out.append(int(lit[i + 1:i + 4], 8))
            i += 4
        else:
            out.append(_ESC[n])
            i += 2
    return bytes(out)


def byte_images(path):
    """Every `data := []byte("..." + "..." ...)` image in a Go test file."""
    src = open(path).read()
    images = []
    for m in re.finditer(r"\[\]byte\(\s*((?:\"(?:[^\"\\]|\\.)*\"\s*\+?\s*)+)\)", src):
        parts = re.findall(r"\"((?:[^\"\\]|\\.)*)\"", m.group(1))
        images.append(b"".join(go_string(p) for p in parts))
    # `crashers := []string{"..." + "...", ...}` (fuzz_test.go)
    for m in re.finditer(r"\[\]string\{((?:\s*(?:\"(?:[^\"\\]|\\.)*\"\s*\+?\s*)+,?)+)\s*\}", src):
        for el in re.finditer(r"((?:\"(?:[^\"\\]|\\.)*\"\s*\+?\s*)+),?", m.group(1)):
            parts = re.findall(r"\"((?:[^\"\\]|\\.)*)\"", el.group(1))
            images.append(b"".join(go_string(p) for p in parts))
    return images


def main(ref):
    os.makedirs(OUT, exist_ok=True)
    k32 = kats(os.path.join(ref, "bitpacking32_test.go"), 32)
    k64 = kats(os.path.join(ref, "bitpacking64_test.go"), 64)
    json.dump({"source": "bitpacking32_test.go unpack8int32Tests", "vectors": k32},
              open(os.path.join(OUT, "bitpack32_kats.json"), "w"))
    json.dump({"source": "bitpacking64_test.go unpack8int64Tests", "vectors": k64},
              open(os.path.join(OUT, "bitpack64_kats.json"), "w"))
    mnc = os.path.join(OUT, "must_not_crash")
    os.makedirs(mnc, exist_ok=True)
    n = 0
    for fn in ["fuzz_test.go", "deltabp_decoder_test.go", "type_dict_test.go", "page_v1_test.go",
               "chunk_reader_test.go", "type_bytearray_test.go", "schema_test.go"]:
        for k, img in enumerate(byte_images(os.path.join(ref, fn))):
            if len(img) < 8:
                continue
            with open(os.path.join(mnc, f"{fn[:-3]}_{k}.bin"), "wb") as f:
                f.write(img)
            n += 1
    print(f"{len(k32)} + {len(k64)} bit-unpack KATs, {n} must-not-crash images")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
