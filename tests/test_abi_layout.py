"""The C ABI's structs as the host binding sees them (swarm_amd/_lib.py ctypes) and as a C
compiler lays them out from include/swarm_hip.h: every size and field offset must agree.
CPU only (gcc on the header; nothing is launched)."""
import ctypes
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ctypes_structs():
    import swarm_amd._lib as L
    return {"swarm_config": L.SwarmConfig, "swarm_replay": L.SwarmReplay, "swarm_act_out": L.SwarmActOut,
            "swarm_adam_cfg": L.SwarmAdamCfg, "swarm_learner": L.SwarmLearner, "swarm_peer": L.SwarmPeer}


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no C compiler")
def test_struct_layouts_match_the_header(tmp_path):
    structs = _ctypes_structs()
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "swarm_hip.h"', "int main(void) {"]
    for name, cls in structs.items():
        lines.append(f'  printf("{name} size %zu\\n", sizeof({name}));')
        for field, _ in cls._fields_:
            lines.append(f'  printf("{name}.{field} %zu\\n", offsetof({name}, {field}));')
    lines.append('  printf("swarm_ctrl size %zu\\n", sizeof(swarm_ctrl));')
    import swarm_amd._lib as L
    for field in L.CTRL:
        lines.append(f'  printf("swarm_ctrl.{field} %zu\\n", offsetof(swarm_ctrl, {field}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                              check=True).stdout.splitlines())
    for name, cls in structs.items():
        assert int(got[f"{name} size"]) == ctypes.sizeof(cls), name
        for field, _ in cls._fields_:
            assert int(got[f"{name}.{field}"]) == getattr(cls, field).offset, f"{name}.{field}"
    import swarm_amd._lib as L
    assert int(got["swarm_ctrl size"]) == 4 * L.CTRL_WORDS
    for field, word in L.CTRL.items():   # the word indices the host reads ctrl by
        assert int(got[f"swarm_ctrl.{field}"]) == 4 * word, field
