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
