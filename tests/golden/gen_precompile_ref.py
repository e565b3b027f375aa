"""Generate tests/golden/precompile_ref.npz: a synthetic block of ed25519-program
instructions (tests/precompile_lib.py random_block, every outcome class) with the
answers of the reference's own fd_precompile_ed25519_verify
(src/flamenco/runtime/program/fd_precompiles.c:120-222), compiled from its source
by oracle/Makefile (_ref/libfdref_precompile.so, driven by oracle/ref_precompile_drv.c).

usage: make -C oracle ref && python tests/golden/gen_precompile_ref.py  (the .npz is committed)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import precompile_lib as P   # noqa: E402


def main():
    pool, desc, tab = P.random_block(4242, 1000)
    err, ce = P.ref_many(pool, desc, tab)
    np.savez_compressed(os.path.join(HERE, "precompile_ref.npz"), pool=pool, desc=desc.view(np.uint8),
                        tab=tab.view(np.uint8), err=err, custom_err=ce)
    print("instructions", desc.size, "outcomes", {int(k): int((ce == k).sum()) for k in np.unique(ce)})


if __name__ == "__main__":
    main()
