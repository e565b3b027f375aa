"""CPU: the frag layouts include/fd_verify_hip.h hard-codes (fd_txn_m_t,
the gossip vote update message, fd_txn_t alignment, FD_TPU_RAW_MTU and the
in-link / tag constants) are the reference's own, checked by compiling the
reference headers (src/disco/fd_txn_m.h, src/flamenco/gossip/fd_gossip_types.h)
next to the engine header with _Static_assert(offsetof(...)) and the
oracle/Makefile machine flags.  Skipped where /root/reference is absent."""
import os
import subprocess

import pytest

from test_ref_boundary import MACHINE, REF_SRC, REPO

SRC = r"""
#include "disco/fd_txn_m.h"
#include "flamenco/gossip/fd_gossip_types.h"
#include "fd_verify_hip.h"
#include <stddef.h>
#define EQ( a, b ) _Static_assert( (a) == (b), #a " != " #b )
EQ( sizeof(fd_txn_m_t),                                   FD_VERIFY_HIP_TXNM_SZ );
EQ( offsetof(fd_txn_m_t, payload_sz),                     FD_VERIFY_HIP_TXNM_PAYLOAD_SZ_OFF );
EQ( offsetof(fd_txn_m_t, txn_t_sz),                       FD_VERIFY_HIP_TXNM_TXN_T_SZ_OFF );
EQ( offsetof(fd_txn_m_t, source_ipv4),                    FD_VERIFY_HIP_TXNM_SRC_IPV4_OFF );
EQ( offsetof(fd_txn_m_t, source_tpu),                     FD_VERIFY_HIP_TXNM_SRC_TPU_OFF );
EQ( offsetof(fd_txn_m_t, block_engine.bundle_id),         FD_VERIFY_HIP_TXNM_BUNDLE_ID_OFF );
EQ( alignof(fd_txn_t),                                    FD_VERIFY_HIP_TXN_ALIGN );
EQ( FD_TPU_RAW_MTU,                                       FD_VERIFY_HIP_TPU_RAW_MTU );
EQ( FD_TPU_MTU,                                           FD_TXN_HIP_MTU );
EQ( FD_TXN_MAX_SZ,                                        FD_TXN_HIP_MAX_SZ );
EQ( FD_TXN_M_TPU_SOURCE_GOSSIP,                           FD_VERIFY_HIP_TPU_SOURCE_GOSSIP );
EQ( FD_GOSSIP_UPDATE_TAG_VOTE,                            FD_VERIFY_HIP_GOSSIP_UPDATE_TAG_VOTE );
EQ( offsetof(fd_gossip_update_message_t, vote.socket.addr), FD_VERIFY_HIP_GOSSIP_VOTE_ADDR_OFF );
EQ( offsetof(fd_gossip_update_message_t, vote.txn_sz),    FD_VERIFY_HIP_GOSSIP_VOTE_TXN_SZ_OFF );
EQ( offsetof(fd_gossip_update_message_t, vote.txn),       FD_VERIFY_HIP_GOSSIP_VOTE_TXN_OFF );
EQ( sizeof(((fd_gossip_vote_t *)0)->txn),                 FD_TXN_HIP_MTU );
int main( void ) { return 0; }
"""


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_SRC, "disco", "fd_txn_m.h")), reason="/root/reference absent")
def test_frag_layouts_match_reference(tmp_path):
    c = tmp_path / "layout.c"
    c.write_text(SRC)
    r = subprocess.run(["gcc", "-O0"] + MACHINE + ["-w", "-I", REF_SRC, "-I", os.path.join(REPO, "include"), "-c",
                        str(c), "-o", str(tmp_path / "layout.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
