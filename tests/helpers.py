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


FUZZ_SPECIALS = [0, 1, 2, 3, 4, 7, 8, 15, 16, 0x7F, 0x80, 0xFE, 0xFF, 0xFFFF, 0x10000, 0x7FFFFFFF, 0xFFFFFFFF]


def structured_mutations(data, offs, seed, per_value=5):
    """The structured fuzz corpus: per valid blob, `per_value` mutants — a bit flip, a truncation,
    a random byte, a header field (counts / lengths / zlbytes / zltail / zllen / intset width and
    count / encoding bytes) or an element length overwritten with a small / boundary / huge value,
    inserted bytes, swapped bytes.  Returns the mutated blobs (the GPU suite and the host codec
    test share it, so both are held to the oracle on the same inputs)."""
    rng = np.random.default_rng(seed)
    specials = FUZZ_SPECIALS
    blobs = []
    for i in range(len(offs) - 1):
        b = bytes(data[offs[i]:offs[i + 1]])
        for _ in range(per_value):
            m = bytearray(b)
            r = int(rng.integers(0, 7))
            if r == 0 and m:
                m[int(rng.integers(0, len(m)))] ^= 1 << int(rng.integers(0, 8))
            elif r == 1 and m:
                m = m[:int(rng.integers(0, len(m)))]
            elif r == 2 and m:
                m[int(rng.integers(0, len(m)))] = int(rng.integers(0, 256))
            elif r == 3 and len(m) >= 9:   # a header field: bytes 5.. hold counts / lengths / ziplist words
                at = int(rng.integers(5, min(len(m) - 3, 30)))
                m[at:at + 4] = int(specials[int(rng.integers(len(specials)))]).to_bytes(4, "little")
            elif r == 4 and len(m) >= 13:  # an element length field somewhere in the body
                at = int(rng.integers(13, len(m) - 3)) if len(m) > 16 else 5
                m[at:at + 4] = int(specials[int(rng.integers(len(specials)))]).to_bytes(4, "little")
            elif r == 5 and m:
                at = int(rng.integers(0, len(m)))
                m[at:at] = bytes(rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8))
            elif r == 6 and len(m) > 2:
                a, c = (int(x) for x in rng.integers(0, len(m), 2))
                m[a], m[c] = m[c], m[a]
            blobs.append(bytes(m))
    return blobs
