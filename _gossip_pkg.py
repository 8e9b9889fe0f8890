"""Import helper: the package directory name (`gossip-protocol-with-power-law_amd`)
is not a Python identifier, so it is loaded under the module name `gossip_amd`."""
import importlib.util
import os
import sys

PKG_NAME = "gossip_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gossip-protocol-with-power-law_amd")


def load():
    mod = sys.modules.get(PKG_NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    spec.loader.exec_module(mod)
    return mod
