"""Lock-step harness: every `volumeRender` mex call the Python mirror of the MATLAB classes makes
is executed by libvrhip (the product) AND replayed into the oracle's model of the reference
(oracle/oracle.py + oracle/vr_oracle.c); every 'render' result is compared under the SURVEY.md 8c
tolerance.  This is how the parity tests read like MATLAB scripts (examples/example1.m etc.)."""
from __future__ import annotations

import numpy as np

import oracle as O
import volume_renderer_amd.volume_render as vrmod
from volume_renderer_amd.mex import volumeRender as real_volume_render
from conftest import assert_parity


def _ovol(v):
    return O.OVolume(v.Data, int(v.TimeLastUpdate))


class Tee:
    def __init__(self, threads: int = 0):
        self.S = O.OracleSession()
        self.hmap = {}
        self.renders = []  # (product image, oracle f32 image, stats)
        self.threads = threads

    def __call__(self, cmd, *args):
        out = real_volume_render(cmd, *args)
        if cmd == "new":
            self.hmap[int(out)] = self.S.new()
        elif cmd == "delete":
            self.S.delete(self.hmap.pop(int(args[0])))
        elif cmd == "sync_volumes":
            h = self.hmap[int(args[0])]
            nrhs = 1 + len(args)
            vols = [_ovol(v) for v in args[2:5]] + ([_ovol(v) for v in args[5:8]] if nrhs == 9 else [])
            self.S.sync_volumes(h, int(args[1]), *vols, nrhs=nrhs)
        elif cmd in ("render", "render_stereo"):
            h = self.hmap[int(args[0])]
            lights, illum = args[1], args[2]
            if isinstance(lights, (bool, np.bool_)) or isinstance(illum, (bool, np.bool_)):
                L, I = None, None
            else:
                seq = lights if isinstance(lights, (list, tuple)) else [lights]
                L = np.array([list(l.Position) + list(l.Color) for l in seq], dtype=np.float32).reshape(-1, 6)
                I = _ovol(illum)
            rest = list(args[3:10])
            if cmd == "render":
                views = [(out, rest)]
            else:  # the fused pair is the reference's two renders: right (+base), then left (-base)
                base = np.float32(args[10])
                left, right = out
                views = []
                for img, off in ((right, base), (left, -base)):
                    props = np.array(rest[4], dtype=np.float32).reshape(-1).copy()  # [xoff f dist]
                    props[0] = off
                    views.append((img, rest[:4] + [props] + rest[5:]))
            for img, r in views:
                # the f32 oracle mutates the session exactly like the product (light upload);
                # the f64 envelope run repeats the same marshalling on the same state.
                ref32, _ = self.S.render(h, L, I, *r, threads=self.threads)
                ref64, _ = self.S.render(h, L, I, *r, double=True, threads=self.threads)
                stats = assert_parity(img, ref32, ref64, what=f"render #{len(self.renders)}")
                self.renders.append((img, ref32, stats))
        return out


def install(monkeypatch, threads: int = 0) -> Tee:
    tee = Tee(threads)
    monkeypatch.setattr(vrmod, "volumeRender", tee)
    return tee
