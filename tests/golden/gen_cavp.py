"""Extract the reference's SHA-512 CAVP vectors into tests/golden/sha512_cavp.npz.

Source (data, not code): /root/reference/src/ballet/sha512/cavp/SHA512ShortMsg.rsp
and SHA512LongMsg.rsp -- the NIST CAVS 11.0 byte-oriented vectors the reference's
test_sha512.c runs.  Every "Len / Msg / MD" record is kept: messages back to back
in one pool (+16 zero bytes of read padding), offsets, byte lengths, digests.

usage: python tests/golden/gen_cavp.py  (needs /root/reference; the .npz is committed)
"""
import os

import numpy as np

SRC = "/root/reference/src/ballet/sha512/cavp"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sha512_cavp.npz")


def parse(path):
    recs, cur = [], {}
    for line in open(path):
        line = line.strip()
        if "=" not in line or line.startswith("#") or line.startswith("["):
            continue
        k, v = (x.strip() for x in line.split("=", 1))
        cur[k] = v
        if k == "MD":
            nbits = int(cur["Len"])
            assert nbits % 8 == 0
            msg = bytes.fromhex(cur["Msg"])[:nbits // 8]
            recs.append((msg, bytes.fromhex(cur["MD"])))
            cur = {}
    return recs


def main():
    pool, off, ln, md, src = bytearray(), [], [], [], []
    for i, name in enumerate(("SHA512ShortMsg.rsp", "SHA512LongMsg.rsp")):
        for msg, d in parse(os.path.join(SRC, name)):
            off.append(len(pool)); ln.append(len(msg)); md.append(np.frombuffer(d, np.uint8)); src.append(i)
            pool += msg
    pool += bytes(16)
    np.savez_compressed(OUT, pool=np.frombuffer(bytes(pool), np.uint8), off=np.array(off, np.uint32),
                        len=np.array(ln, np.uint32), md=np.stack(md), src=np.array(src, np.uint8))
    print(f"{len(off)} vectors ({sum(1 for s in src if s == 0)} short, {sum(1 for s in src if s == 1)} long), "
          f"{len(pool)} pool bytes -> {OUT}")


if __name__ == "__main__":
    main()
