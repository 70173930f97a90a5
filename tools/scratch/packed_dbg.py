import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "minesweeper-ppo_amd"))
import numpy as np, torch
from ms_amd import EnvConfig, VecMinesweeper, _lib as L
for (H, W, K) in ((8, 8, 10), (9, 9, 10)):
    N = 64
    a = VecMinesweeper(N, EnvConfig(H=H, W=W, mine_count=K), seed=0)
    b = VecMinesweeper(N, EnvConfig(H=H, W=W, mine_count=K), seed=0)
    b.set_debug_flags(L.MS_DBG_ONE_BOARD_PER_WAVE)
    a.reset(); b.reset()
    bad = 0
    for t in range(6):
        act = a.tape_actions(t, 0)
        sa0 = a.snapshot_tensors()
        a.step(act); b.step(act)
        ma = a.snapshot_tensors()["mine"].cpu().numpy().reshape(N, -1)
        mb = b.snapshot_tensors()["mine"].cpu().numpy().reshape(N, -1)
        for e in np.nonzero((ma != mb).any(1))[0][:3]:
            print(H, W, "t", t, "env", e, "click", int(act[e]), "packed", np.nonzero(ma[e])[0].tolist(), "ref", np.nonzero(mb[e])[0].tolist())
            bad += 1
    print(H, W, "mismatching env-steps:", bad, "rng equal:", np.array_equal(a.rng_state(), b.rng_state()))
