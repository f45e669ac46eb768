import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP library)')


@pytest.fixture(scope='session')
def scene_dir(tmp_path_factory):
    """Deterministic data.bin files for every named scene."""
    from swift3drenderer_amd import scene
    d = tmp_path_factory.mktemp('scenes')
    paths = {}
    for name in ('full', 'flat', 'tetra', 'regular'):
        p = str(d / f'{name}.bin')
        scene.write_named(name, p)
        paths[name] = p
    return paths


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope='session')
def gpu_renderer():
    if not gpu_available():
        pytest.skip('no GPU')
    from swift3drenderer_amd.renderer import Renderer
    return Renderer()


@pytest.fixture(autouse=True)
def _gpu_output_uncaptured(request):
    """GPU tests run with pytest's fd capture off: a library that ends the process (a device fault's
    HIPCHECK abort, a bounded wait's stall exit) prints its reason to stderr first, and a captured
    stderr dies with the process -- the round-4 aborts lost their messages that way."""
    if request.node.get_closest_marker('gpu') is None:
        yield
        return
    capman = request.config.pluginmanager.getplugin('capturemanager')
    if capman is None:
        yield
        return
    with capman.global_and_fixture_disabled():
        yield
