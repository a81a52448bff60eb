"""Load the reference MLIC++ models (read-only /root/reference) on CPU through the
compressai/timm test shim in oracle/refshim.  Used ONLY by oracle/gen_golden.py in
this container to produce tests/golden fixtures; /root/reference does not exist on
the GPU box and nothing at run time imports this file."""
import importlib.util
import os
import sys

REF = os.environ.get("MLIC_REFERENCE", "/root/reference/MLIC++")
_HERE = os.path.dirname(os.path.abspath(__file__))


def _setup():
    sys.dont_write_bytecode = True
    shim = os.path.join(_HERE, "refshim")
    for p in (REF, shim):
        if p not in sys.path:
            sys.path.insert(0, p)


def load_module(rel):
    _setup()
    name = "mlicref_" + rel.replace("/", "_").replace(".py", "")
    if name in sys.modules:
        return sys.modules[name]
    sp = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(sp)
    sys.modules[name] = mod
    sp.loader.exec_module(mod)
    return mod


class _Cfg(dict):
    __getattr__ = dict.__getitem__


def build(name):
    """Instantiate the reference class for model `name` (eval mode, CPU)."""
    import torch.nn as nn
    from mlic_amd import spec
    cfg = spec.get_config(name)
    c = _Cfg(N=cfg.N, M=cfg.M, slice_num=cfg.slice_num, context_window=cfg.context_window, act=nn.GELU)
    if cfg.small_decoder and cfg.vbr:
        cls = load_module("models/mlicpp_sd_vbr.py").MLICPlusPlusSDVbr
    elif cfg.small_decoder:
        cls = load_module("models/mlicpp_small_decoder.py").MLICPlusPlusSD
    elif cfg.vbr:
        cls = load_module("models/mlicpp_vbr.py").MLICPlusPlusVbr
    else:
        cls = load_module("models/mlicpp.py").MLICPlusPlus
    return cls(config=c).eval()
