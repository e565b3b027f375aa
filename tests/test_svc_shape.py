"""The service's segment shape in the reference's topologies (CPU).

integration/fd_verify_topo_hip.patch gives each GPU tile's verify_svc object
the shape fd_verify_svc_topo_shape( tiles that GPU serves ) returns
(include/fd_verify_svc.h).  fd_verify_svc_boot refuses a shape outside the
checks of fd_verify_svc_boot_ok (the same header function: staging below
4 GiB, ingest chunk indices within 32 bits, batch_max at least a slot).  Round
5's fixed shape (16 slots x 32768 frags) could not boot the reference's
default verify_tile_count = 6 on one GPU (6.85 GB of staging; VERDICT r05,
missing #2).

Here every verify_tile_count in 1..16 on 1..8 GPUs, with 0..5 client tiles
(shred tiles, the replay tile: include/fd_verify_svc.h "clients") on GPU 0:
each GPU's shape boots
with the GPU tile's defaults (batch_max 262144, 2 launches in flight,
integration/fd_verify_gpu_tile.c), the shapes cover every verify tile once,
and the staging bound is recomputed here independently of the header."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = r"""
#include <stdio.h>
#include "fd_verify_svc.h"
int main( void ) {
  printf( "{\"rows\": [" );
  int first = 1;
  /* clients on GPU 0 (the topology patch): shred tiles (1..4), plus the
     replay tile in the Firedancer topology */
  for( ulong v=1UL; v<=16UL; v++ ) for( ulong gpus=1UL; gpus<=8UL; gpus++ ) for( ulong cl=0UL; cl<=5UL; cl++ ) {
    ulong gc = gpus<v ? gpus : v;                       /* vgpu_cnt = min( FD_VERIFY_SVC_GPU_CNT, verify_tile_cnt ) */
    for( ulong g=0UL; g<gc; g++ ) {
      ulong sh[ 4 ] = { 0UL, 0UL, 0UL, 0UL };
      int rc = fd_verify_svc_topo_shape( fd_verify_svc_tiles_on( g, v, gc ) + ( g ? 0UL : cl ), sh );
      int ok = !rc && fd_verify_svc_boot_ok( sh[0], sh[1], sh[2], sh[3], 262144UL, 2UL );
      printf( "%s{\"verify\": %lu, \"gpus\": %lu, \"g\": %lu, \"clients\": %lu, \"rc\": %d, \"boot_ok\": %d, "
              "\"shape\": [%lu, %lu, %lu, %lu], \"footprint\": %lu}", first ? "" : ", ", v, gc, g, g ? 0UL : cl, rc, ok,
              sh[0], sh[1], sh[2], sh[3], fd_verify_svc_footprint( sh[0], sh[1], sh[2], sh[3] ) );
      first = 0;
    }
  }
  /* round 5's fixed shape at the default 6 tiles, and a shape just over the bound */
  printf( "], \"r05_6\": %d, \"over\": %d}\n", fd_verify_svc_boot_ok( 6UL, 16UL, 32768UL, 4096UL, 262144UL, 2UL ),
          fd_verify_svc_boot_ok( 6UL, 128UL, 4096UL, 256UL, 262144UL, 2UL ) );
  return 0;
}
"""


@pytest.fixture(scope="module")
def shapes(tmp_path_factory):
    d = tmp_path_factory.mktemp("shape")
    src, exe = d / "shape.c", d / "shape"
    src.write_text(PROG)
    subprocess.check_call(["gcc", "-std=c17", "-O1", "-Wall", "-Werror", "-I" + os.path.join(REPO, "include"),
                           "-o", str(exe), str(src)])
    out = subprocess.check_output([str(exe)], text=True)
    d = json.loads(out)
    return d["rows"], d


def test_every_topology_shape_boots(shapes):
    rows, _ = shapes
    assert len(rows) == 6 * sum(min(g, v) for v in range(1, 17) for g in range(1, 9))
    for r in rows:
        t, depth, cap, frag = r["shape"]
        assert r["rc"] == 0 and r["boot_ok"] == 1, r
        # the service's bounds, recomputed: staging (2176 B a frag) below 4 GiB, ingest (32 chunks a frag)
        # chunk indices below 2^32, the tile's slot array (FD_VERIFY_SVC_SLOT_MAX 256)
        assert t * depth * cap * 2176 + 4096 < 1 << 32, r
        assert 32 * t * depth * cap < 1 << 32 and depth <= 256 and frag <= cap and r["footprint"] > 0, r


def test_shapes_cover_every_tile(shapes):
    rows, _ = shapes
    for v in range(1, 17):
        for gpus in range(1, 9):
            for cl in range(6):
                sel = [r for r in rows if r["verify"] == v and r["gpus"] == min(gpus, v) and
                       (r["g"] > 0 or r["clients"] == cl)]
                by_g = {r["g"]: r["shape"][0] - r["clients"] for r in sel}
                served = list(by_g.values())
                assert len(served) == min(gpus, v) and sum(served) == v and max(served) - min(served) <= 1, (v, gpus, served)
                assert {r["shape"][0] for r in sel if r["g"] == 0} == {by_g[0] + cl}


def test_reference_default_six_tiles_on_one_gpu(shapes):
    """verify_tile_count = 6 (src/app/fdctl/config/default.toml:776) on one GPU:
    128 slots of 2048 frags (3.4 GB of staging); round 5's 16 x 32768 does not
    boot, and twice the slot capacity is over the bound"""
    rows, extra = shapes
    six = [r for r in rows if r["verify"] == 6 and r["gpus"] == 1 and r["clients"] == 0]
    assert six and six[0]["shape"] == [6, 128, 2048, 256]
    # with the Firedancer topology's clients on GPU 0 (one shred tile, the replay tile): 8 tiles, 1024-frag slots
    eight = [r for r in rows if r["verify"] == 6 and r["gpus"] == 1 and r["clients"] == 2]
    assert eight and eight[0]["shape"] == [8, 128, 1024, 256] and eight[0]["boot_ok"] == 1
    assert extra["r05_6"] == 0 and extra["over"] == 0
