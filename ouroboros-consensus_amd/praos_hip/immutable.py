"""ImmutableDB directories of synthetic chains (db-synthesizer analogue) for the replay
driver (praos_replay_immutable).

On-disk layout written (ouroboros-consensus Storage/ImmutableDB/Impl):
  NNNNN.chunk      the stored blocks of chunk N back to back (chunk.pack_chunk layout:
                   [6, [header, [], [], {}, []]]);
  NNNNN.secondary  one 56-byte big-endian Entry per block (Index/Secondary.hs:93-128):
                   blockOffset u64, headerOffset u16, headerSize u16, checksum u32
                   (CRC32 of the block bytes), headerHash 32, blockOrEBB = slot u64;
  NNNNN.primary    version byte 1, then u32 BE secondary offsets, one per relative slot
                   plus one (Index/Primary.hs:104-160; relative slot 0 is the EBB slot).
A block of slot s lives in chunk s // chunk_slots (ChunkInfo with a uniform chunk size).

make_multi_epoch_chain forges a linked chain across several epochs: per epoch the
first-leader-wins schedule under that epoch's nonce (praos_leader_schedule), signed
with hbPrev = headerHash of the previous block and consecutive block numbers, and the
next epoch nonce taken from the chain state folded over the epoch (tickChainDepState:
candidate ⭒ lastEpochBlock, Praos.hs:407-431).
"""
import hashlib
import os
import zlib

import numpy as np

from . import chains
from .chunk import HEADER_OFFSET, pack_chunk

ENTRY = 56


def write_immutable(path, arena, off, length, slots, header_hash, chunk_slots):
    """arena/off/length: pack_chunk output (off/length = the headers inside their blocks).
    Returns the number of chunk files written."""
    os.makedirs(path, exist_ok=True)
    n = len(off)
    slots = np.asarray(slots, np.uint64)
    bstart = off.astype(np.int64) - HEADER_OFFSET
    bend = np.append(bstart[1:], len(arena)) if n else bstart
    chunk_of = (slots // np.uint64(chunk_slots)).astype(np.int64)
    last = int(chunk_of[-1]) if n else -1
    for c in range(last + 1):
        rows = np.nonzero(chunk_of == c)[0]
        data, sec = bytearray(), bytearray()
        prim = [0] * (chunk_slots + 2)
        for i in rows:
            blk = arena[bstart[i]:bend[i]].tobytes()
            sec += (len(data).to_bytes(8, "big") + HEADER_OFFSET.to_bytes(2, "big") +
                    int(length[i]).to_bytes(2, "big") + zlib.crc32(blk).to_bytes(4, "big") +
                    bytes(header_hash[i]) + int(slots[i]).to_bytes(8, "big"))
            data += blk
            rel = 1 + int(slots[i]) - c * chunk_slots        # relative slot (0 = EBB)
            prim[rel + 1] = len(sec)
        for k in range(1, len(prim)):                        # empty slots repeat the offset
            prim[k] = max(prim[k], prim[k - 1])
        with open(os.path.join(path, f"{c:05d}.chunk"), "wb") as f:
            f.write(data)
        with open(os.path.join(path, f"{c:05d}.secondary"), "wb") as f:
            f.write(sec)
        with open(os.path.join(path, f"{c:05d}.primary"), "wb") as f:
            f.write(b"\x01" + b"".join(x.to_bytes(4, "big") for x in prim))
    return last + 1


def read_secondary(path, chunk):
    """Entries of one secondary index as a list of dicts (for tests and tools)."""
    raw = open(os.path.join(path, f"{chunk:05d}.secondary"), "rb").read()
    out = []
    for k in range(0, len(raw), ENTRY):
        e = raw[k:k + ENTRY]
        out.append({"block_offset": int.from_bytes(e[0:8], "big"), "header_offset": int.from_bytes(e[8:10], "big"),
                    "header_size": int.from_bytes(e[10:12], "big"), "checksum": int.from_bytes(e[12:16], "big"),
                    "header_hash": e[16:48], "slot": int.from_bytes(e[48:56], "big")})
    return out


def _combine(a, b):
    if a is None:
        return b
    if b is None:
        return a
    return hashlib.blake2b(a + b, digest_size=32).digest()


def make_multi_epoch_chain(ctx, cfg, epochs, epoch_length, stability_window, tpraos=False, extra_entropy=None,
                           progress=None, schedules=None, stakes=None):
    """A linked chain over `epochs` epochs of `epoch_length` slots from slot 0 (Origin,
    GenesisHash, epoch 0 nonce = cfg["eta0"]).  Returns dict(arena, off, len, slots,
    header_hash, pools, params, nonces (per epoch), state (after the last
    block, as Context.update_chain_dep_state keeps it)).  tpraos=True: a Shelley..Alonzo
    chain (TPraos leader schedule and BHeaders, stored as Alonzo blocks, era tag 5; the
    TPraos nonce rules with TICKN's extra_entropy).  schedules: {epoch: (slots, pools)} used
    instead of the leader-schedule search for those epochs (e.g. epoch 0 of the C5 / tp chain
    from its shipped schedule, which was searched under the same seed, stake and nonce).
    stakes: a function epoch -> per-pool Fixed E34 stake (0 = the pool is not in that epoch's
    PoolDistr), so the stake distribution changes between epochs as the ledger's NEWEPOCH makes
    it (the leader schedule of epoch e is searched under epoch e's stake); the result then has
    "views": [(epoch, pool list)] -- the LedgerView's PoolDistr per epoch."""
    sig0 = chains.stake(cfg["npools"], cfg["stake_offset"])
    views, used = [], []
    p = chains.params(cfg)
    st = {"last_slot": None, "counters": {}, "evolving": cfg["eta0"], "candidate": cfg["eta0"],
          "epoch_nonce": cfg["eta0"], "lab": None, "leb": None}
    ei = (0, 0, epoch_length, stability_window)
    eta = cfg["eta0"]
    parts, nonces, slots_all, hh_all = [], [], [], []
    prev, block_no, pool_list = None, 0, None
    for e in range(epochs):
        if e > 0:
            eta = _combine(st["candidate"], st["leb"])      # the tick into epoch e
            if tpraos:
                eta = _combine(eta, extra_entropy)          # TICKN
        nonces.append(eta)
        sig = list(stakes(e)) if stakes else sig0
        if schedules and e in schedules:
            sl, pl = schedules[e]
            keep = (sl >= e * epoch_length) & (sl < (e + 1) * epoch_length)
            sl, pl = sl[keep].astype(np.uint64), pl[keep].astype(np.uint32)
        elif cfg.get("round_robin"):
            # f = 1 (every pool a leader in every slot, checkLeaderNatValue's f == 1 case):
            # a block in every slot, forged by the pools in turn -- a dense chain of the C5
            # shape (432k headers per 432k-slot epoch) without the 26e9-evaluation search
            assert cfg["f"] == 1, "round_robin schedules are leader-valid only for f = 1"
            sl = np.arange(e * epoch_length, (e + 1) * epoch_length, dtype=np.uint64)
            pl = (sl % cfg["npools"]).astype(np.uint32)
        else:
            lead = ctx.leader_schedule(cfg["seed"], sig, p, eta, e * epoch_length, epoch_length, tpraos=tpraos)
            idx = np.nonzero(lead >= 0)[0]
            sl = (e * epoch_length + idx).astype(np.uint64)
            pl = lead[idx].astype(np.uint32)
        n = len(sl)
        used.append((sl, pl))
        H, keys, _ = ctx.synthesize(n, cfg["npools"], p, eta, cfg["seed"], body_len=0, schedule=(sl, pl),
                                    block_no0=block_no, link=True, prev0=prev, tpraos=tpraos)
        pool_list = [(h, v, s) for (h, v), s in zip(keys, sig) if s > 0]
        views.append((e, pool_list))
        # fold the clean chain to learn the next nonce (the generator's own ledger)
        ctx.set_epoch(eta, pool_list, p)
        o = ctx.verify_tpraos_headers(H) if tpraos else ctx.verify_headers(H)
        prev_hash = np.zeros((n, 32), np.uint8)
        gen = np.zeros(n, np.uint8)
        if prev is None:
            gen[0] = 1
        else:
            prev_hash[0] = np.frombuffer(prev, np.uint8)
        prev_hash[1:] = H["header_hash"][:-1]
        if tpraos:
            _, _, stop, _ = ctx.tpraos_update_chain_dep_state(H, o, prev_hash, st, ei, prev_is_genesis=gen,
                                                              extra_entropy=extra_entropy)
        else:
            _, stop, _ = ctx.update_chain_dep_state(H, o, prev_hash, st, ei, prev_is_genesis=gen)
        if stop != n:
            raise RuntimeError(f"epoch {e}: generated header {stop} does not validate")
        parts.append(H)
        slots_all.append(sl)
        hh_all.append(H["header_hash"])
        prev = bytes(H["header_hash"][-1])
        block_no += n
        if progress:
            progress(e, n)
    # one stored-bytes arena over all epochs
    arenas, offs, lens, base = [], [], [], 0
    for H in parts:
        a, o_, l_ = pack_chunk(H, era_tag=5 if tpraos else 6)
        arenas.append(a)
        offs.append(o_ + np.uint64(base))
        lens.append(l_)
        base += len(a)
    return {"arena": np.concatenate(arenas), "off": np.concatenate(offs), "len": np.concatenate(lens),
            "slots": np.concatenate(slots_all), "header_hash": np.concatenate(hh_all), "pools": pool_list,
            "params": p, "nonces": nonces, "state": st,
            "epoch_info": ei, "views": views, "schedules": used}
