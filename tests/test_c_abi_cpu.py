"""CPU side of the C-ABI harness: the binary exists after the build and links against the
in-tree product library and the oracle (no GPU needed to check the link)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "c_abi", "abi_parity")


def test_c_abi_harness_links_in_tree_libraries():
    from f16_jsb_amd.build import build
    from oracle_ref import build_oracle
    build()          # the product library and the oracle the harness links (no-ops when current)
    build_oracle()
    subprocess.run(["make", "-C", os.path.join(HERE, "c_abi")], check=True, capture_output=True)
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, check=True).stdout
    lines = {l.split()[0]: l for l in out.splitlines() if "=>" in l}
    root = os.path.dirname(HERE)
    assert os.path.realpath(lines["libf16env.so"].split("=>")[1].split("(")[0].strip()) == \
        os.path.realpath(os.path.join(root, "f16_jsb_amd", "libf16env.so"))
    assert "libf16ref.so" in lines and "not found" not in out
