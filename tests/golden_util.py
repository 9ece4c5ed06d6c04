"""Helpers to read the committed reference fixtures (tests/golden/*.json).

The fixtures were produced by oracle/gen_golden.c driving the reference
(cisco/libsrtp built from its sources, oracle/Makefile.ref); see
tests/golden/README.md.
"""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def all_cases():
    out = []
    for f in ("ref_int.json", "ref_ossl.json"):
        for c in load(f)["cases"]:
            out.append(c)
    return out


def case_ids():
    return [c["name"] for c in all_cases()]
