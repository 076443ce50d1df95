"""Tools only: the diagnostic environment variables of earlier rounds mapped onto kp_overrides (ABI v12). libkp itself
reads no environment variable; a tool calls apply(ctx) after creating its context."""
import os

ENV = {"KP_TIMING": ("timing", lambda v: 1), "KP_HOST_TIMING": ("host_timing", lambda v: 1),
       "KP_CONT": ("fast_lane", lambda v: 2 if v not in ("", "0") else 1),
       "KP_SORT_CAP": ("sort_capacity", int), "KP_CHK_MAXC": ("chunk_capacity", lambda v: int(v) if int(v) else -1),
       "KP_NO_TFEAS": ("template_table", lambda v: 1), "KP_GENERAL_BATCH": ("general_batch", lambda v: 1 if v == "0" else 0),
       "KP_FEAS_GLOBAL": ("feasibility_kernel", lambda v: 1), "KP_FEAS_ONE_ROW": ("feasibility_kernel", lambda v: 2),
       "KP_FEAS_BLOCKS": ("feasibility_blocks", int), "KP_FEAS_TEMPORAL": ("feasibility_temporal", lambda v: 1),
       "KP_TFEAS_SHARD_MIN": ("table_shard_min", lambda v: max(1, int(v)))}


def apply(ctx, env=None):
    """ctx.set_overrides from the variables present; a libkp build older than ABI v12 (tools' A/B builds) has no
    kp_ctx_set_overrides and reads the variables itself."""
    env = os.environ if env is None else env
    kw = {f: conv(env[k]) for k, (f, conv) in ENV.items() if k in env}
    if getattr(ctx.lib, "kp_ctx_set_overrides", None) is not None:
        ctx.set_overrides(**kw)
    return kw
