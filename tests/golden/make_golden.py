#!/usr/bin/env python3
"""Extract known-answer vectors from the reference's own golden files.

Run in the build container (needs /root/reference; the GPU box never does):
    python tests/golden/make_golden.py
Writes tests/golden/reference_kats.json (data only: inputs + expected
outputs).  The reference itself is Haskell and cannot run here; these blocks
were produced by its example generator with real StandardCrypto keys
(ouroboros-consensus-cardano/src/shelley-testlib/Test/Consensus/Shelley/
Examples.hs:74-256) and are compared byte-for-byte by its golden tests
(consensus-testlib/Test/Util/Serialisation/Golden.hs:102-121), so the
signatures and VRF outputs in them are reference outputs.

Expected values and where they come from:
  * OCert Ed25519 over hotVK||BE64(n)||BE64(c0) is valid in every block
    (the example signs it with the cold key).
  * TPraos blocks (Shelley..Alonzo): Sum6KES at t=0 over the raw 15-field
    BHBody is valid; the two VRF certs (eta, leader) verify for
    alpha = Blake2b256(0x00) / Blake2b256(0x01) (the example's dummy seeds),
    and the stored 64-B outputs equal proof_to_hash.
  * Every block matches its header (blockMatchesHeader): the header body hash
    is the reference's hashTxSeq of the stored block segments.
  * Praos blocks (Babbage, Conway): Examples.hs:173-192 coerce the TPraos KES
    signature into the Praos header, so the Merkle path is valid but the leaf
    signature does NOT verify over the 10-field Praos body (a natural
    InvalidKesSignatureOCERT vector); it does verify over the Shelley 15-field
    body with the Praos block's body hash substituted (reconstructed here).
    The Praos VRF cert is the TPraos eta cert (alpha = Blake2b256(0x00)).
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import cbor_min  # noqa: E402

REF = "/root/reference/ouroboros-consensus-cardano/golden"
FILES = {
    "Shelley": "cardano/disk/Block_Shelley",
    "Allegra": "cardano/disk/Block_Allegra",
    "Mary": "cardano/disk/Block_Mary",
    "Alonzo": "cardano/disk/Block_Alonzo",
    "ShelleyOnly": "shelley/disk/Block",
    "Babbage": "cardano/disk/Block_Babbage",
    "Conway": "cardano/disk/Block_Conway",
}


def b2b(m, n=32):
    return hashlib.blake2b(m, digest_size=n).digest()


def header_of(buf):
    it = cbor_min.decode(buf)
    v = it.value
    blk = v[1] if (len(v) == 2 and isinstance(v[0].value, int)) else it
    return blk.value[0]


def main():
    kats = []
    shelley_body = None
    for era, rel in FILES.items():
        path = os.path.join(REF, rel)
        buf = open(path, "rb").read()
        h = header_of(buf)
        body_it, sig_it = h.value
        f = body_it.value
        body = body_it.raw(buf)
        rec = {"era": era, "file": "ouroboros-consensus-cardano/golden/" + rel,
               "header_cbor": h.raw(buf).hex(), "body_cbor": body.hex(),
               "kes_sig": sig_it.value.hex(),
               # the whole stored block (HardForkBlock [eraTag, block] or a bare Shelley block):
               # the block-integrity batch (Integrity.hs:14-20) hashes its segments
               "block_cbor": buf.hex()}
        if len(f) == 15:  # TPraos BHBody (cardano-protocol-tpraos BHeader)
            rec.update(kind="tpraos", block_no=f[0].value, slot=f[1].value,
                       cold_vk=f[3].value.hex(), vrf_vk=f[4].value.hex(),
                       eta_out=f[5].value[0].value.hex(), eta_proof=f[5].value[1].value.hex(),
                       leader_out=f[6].value[0].value.hex(), leader_proof=f[6].value[1].value.hex(),
                       body_hash=f[8].value.hex(), hot_vk=f[9].value.hex(), n=f[10].value,
                       c0=f[11].value, ocert_sig=f[12].value.hex())
            rec["expect"] = {"ocert_valid": True, "kes_t": 0, "kes_result": 0,
                             "eta_alpha": b2b(b"\x00").hex(), "eta_valid": True,
                             "leader_alpha": b2b(b"\x01").hex(), "leader_valid": True}
            if era == "Shelley":
                shelley_body = (body, f[8])
        else:  # Praos HeaderBody, Header.hs:168-193
            vr = f[5].value
            oc = f[8].value
            rec.update(kind="praos", block_no=f[0].value, slot=f[1].value,
                       cold_vk=f[3].value.hex(), vrf_vk=f[4].value.hex(),
                       vrf_out=vr[0].value.hex(), vrf_proof=vr[1].value.hex(),
                       body_size=f[6].value, body_hash=f[7].value.hex(),
                       hot_vk=oc[0].value.hex(), n=oc[1].value, c0=oc[2].value, ocert_sig=oc[3].value.hex(),
                       prot=[f[9].value[0].value, f[9].value[1].value])
            # the TPraos body the KES leaf was really made over
            rec["_note"] = "kes_recon_body = Shelley BHBody with this block's body_hash"
            rec["expect"] = {"ocert_valid": True, "kes_t": 0, "kes_merkle_ok": True,
                             "kes_result_praos_body": 2,
                             "vrf_alpha": b2b(b"\x00").hex(), "vrf_valid": True}
            recon_body = reconstruct(shelley_body, bytes.fromhex(rec["body_hash"]))
            rec["kes_recon_body"] = recon_body.hex()
            rec["expect"]["kes_result_recon_body"] = 0
        # blockMatchesHeader (Shelley/Ledger/Block.hs:150-158): the stored header's body hash
        # is the reference's hashTxSeq of these segments -- every golden block matches
        rec["expect"]["block_matches_header"] = True
        kats.append(rec)
    out = os.path.join(HERE, "reference_kats.json")
    with open(out, "w") as fh:
        json.dump({"source": "karknu/ouroboros-consensus golden blocks (see make_golden.py)",
                   "kats": kats}, fh, indent=1)
    print("wrote", out, len(kats), "vectors")


def reconstruct(shelley_body, body_hash: bytes) -> bytes:
    """Shelley 15-field BHBody bytes with field 8 (bhash) replaced."""
    body, hash_item = shelley_body
    # locate the 32-byte hash payload inside the raw body bytes
    old = hash_item.value
    i = body.find(b"\x58\x20" + old)
    assert i >= 0
    return body[:i + 2] + body_hash + body[i + 2 + 32:]


if __name__ == "__main__":
    main()
