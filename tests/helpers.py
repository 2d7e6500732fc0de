"""Shared test helpers: golden fixtures, batch assembly and flat-form comparison."""
import json
import os

import numpy as np

import redrock_old_amd as rr

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat.json")


def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def batch_from_blobs(blobs):
    """Concatenate blobs into (data padded to 16, offsets)."""
    offs = np.zeros(len(blobs) + 1, np.uint64)
    for i, b in enumerate(blobs):
        offs[i + 1] = offs[i] + len(b)
    raw = b"".join(blobs)
    pad = (len(raw) + 15) & ~15
    data = np.zeros(pad, np.uint8)
    data[:len(raw)] = np.frombuffer(raw, np.uint8) if raw else data[:0]
    return data, offs


def expected_flat(fixtures):
    """Expected (values, elems) for a batch made of the fixtures in order."""
    values = np.zeros(len(fixtures), rr.VALUE_DT)
    elems = []
    off = 0
    for i, fx in enumerate(fixtures):
        blob = bytes.fromhex(fx["blob"])
        v = fx["value"]
        values[i]["type"] = blob[0] if blob else 0
        values[i]["enc"] = v["enc"]
        values[i]["lru"] = v["lru"]
        values[i]["status"] = v.get("status", 0)
        values[i]["n_elems"] = len(fx["elems"]) if v.get("status", 0) == 0 else 0
        values[i]["elem_base"] = len(elems)
        for kind, data, ln, zenc in fx["elems"]:
            d = data + off if kind in (rr.K_STR, rr.K_ZLRAW) else data
            elems.append((d & 0xFFFFFFFFFFFFFFFF, ln, kind, zenc, 0))
        # a malformed value keeps its reserved slots zero-filled; so does the unused tail of a
        # de-duplicated set
        used = len(fx["elems"]) if v.get("status", 0) == 0 else 0
        elems.extend([(0, 0, 0, 0, 0)] * (v.get("reserve", used) - used))
        off += len(blob)
    return values, np.array(elems, dtype=rr.ELEM_DT)


def assert_flat_equal(a, b, what=""):
    (va, ea), (vb, eb) = a, b
    if not np.array_equal(va, vb):
        bad = np.nonzero(va != vb)[0]
        i = int(bad[0])
        raise AssertionError(f"{what}: {len(bad)} value records differ; first #{i}: {va[i]} vs {vb[i]}")
    if len(ea) != len(eb) or not np.array_equal(ea, eb):
        n = min(len(ea), len(eb))
        bad = np.nonzero(ea[:n] != eb[:n])[0]
        i = int(bad[0]) if len(bad) else n
        raise AssertionError(f"{what}: descriptors differ (len {len(ea)} vs {len(eb)}); first #{i}: "
                             f"{ea[i] if i < len(ea) else None} vs {eb[i] if i < len(eb) else None}")
