"""Schedule tuning for the development tools: ARTES_<KEY> environment variables (the knobs of
earlier rounds' A/B scripts) applied to a grid handle through artes_set_tuning.  The
production library reads no environment variable itself (include/artes_amd.h)."""
import os

from artes_amd.engine import TUNING_KEYS


def env_tuning(env=None) -> dict:
    env = os.environ if env is None else env
    out = {}
    for k in TUNING_KEYS:
        v = env.get("ARTES_" + k.upper())
        if v is not None:
            out[k] = v if k == "engine" else int(v)
    return out


def apply(grid, env=None) -> dict:
    """Set what the handle accepts; a key it rejects (e.g. steps=4 on a radial-only grid) is
    reported and left at its default."""
    from artes_amd.engine import EngineError

    kv, done = env_tuning(env), {}
    for k, v in kv.items():
        try:
            grid.set_tuning(**{k: v})
            done[k] = v
        except EngineError as e:
            print(f"[tuning] {k}={v} not applied: {e}", flush=True)
    return done
