"""TEST TOOLING ONLY (build container): copies the lib0 payload vectors of
yrs/src/tests/compatibility_tests.rs (map_set, array_insert, xml_fragment_insert:
v1 + v2 pairs of the same blocks; utf32_lib0_v2_decoding: a v2 update) into
tests/golden/compat_v2.json (data only)."""
import json
import os
import re

SRC = "/root/reference/yrs/src/tests/compatibility_tests.rs"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    src = open(SRC).read()
    vecs = []
    for m in re.finditer(r"let (payload|data)\s*=\s*&\[(.*?)\];", src, re.S):
        line = src[:m.start()].count("\n") + 1
        vecs.append((line, bytes(int(x) for x in re.findall(r"\d+", m.group(2)))))
    by_line = dict(vecs)
    out = {
        "source": "yrs/src/tests/compatibility_tests.rs",
        "pairs": {  # name: [v1 payload (line), v2 payload (line)] — roundtrip_v1 / roundtrip_v2 of one block list
            "map_set": [by_line[178].hex(), by_line[184].hex()],
            "array_insert": [by_line[220].hex(), by_line[225].hex()],
            "xml_fragment_insert": [by_line[277].hex(), by_line[284].hex()],
        },
        "utf32_lib0_v2_decoding": by_line[322].hex(),
    }
    with open(os.path.join(ROOT, "tests", "golden", "compat_v2.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
