#!/usr/bin/env python3
"""Extract the PraosState encodings from the reference's golden ChainDepState files
(ouroboros-consensus-cardano/golden/cardano/disk/ChainDepState_{Babbage,Conway}:
the hard-fork telescope's current era = [bound, PraosState]) into
tests/golden/praos_state.json: the raw bytes of the Praos.hs:274-310 encoding and the
values it holds.  Run in this container (the reference tree is not on the GPU box)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import cbor_min as c  # noqa: E402

REF = "/root/reference/ouroboros-consensus-cardano/golden/cardano/disk"


def _nonce(it):
    v = it.value
    return None if v[0].value == 0 else v[1].value.hex()


def main():
    out = []
    for era in ("Babbage", "Conway"):
        d = open(os.path.join(REF, f"ChainDepState_{era}"), "rb").read()
        cur = c.decode(d).value[-1]             # current era of the telescope: [bound, state]
        st = cur.value[1]
        raw = st.raw(d)
        ver, body = st.value[0].value, st.value[1].value
        ls = body[0].value
        counters = body[1].value
        pairs = counters.items() if isinstance(counters, dict) else counters
        out.append({"era": era, "source": f"golden/cardano/disk/ChainDepState_{era} bytes {st.start}..{st.end}",
                    "cbor": raw.hex(), "version": ver,
                    "last_slot": None if ls[0].value == 0 else ls[1].value,
                    "counters": {k.value.hex(): v.value for k, v in pairs},
                    "evolving": _nonce(body[2]), "candidate": _nonce(body[3]), "epoch_nonce": _nonce(body[4]),
                    "lab": _nonce(body[5]), "leb": _nonce(body[6])})
    json.dump({"generator": "tests/golden/make_state_golden.py", "states": out},
              open(os.path.join(HERE, "praos_state.json"), "w"), indent=1)
    print(json.dumps(out, indent=1)[:1500])


if __name__ == "__main__":
    main()
