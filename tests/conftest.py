import importlib
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, os.path.join(REPO, "oracle"), GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def Q():
    return importlib.import_module("incubator-druid_amd.query")


@pytest.fixture(scope="session")
def W():
    return importlib.import_module("incubator-druid_amd.writer")


@pytest.fixture(scope="session")
def DG():
    return importlib.import_module("incubator-druid_amd.datagen")


@pytest.fixture(scope="session")
def O():
    import oracle
    return oracle


@pytest.fixture(scope="session")
def kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def engine_kats():
    with open(os.path.join(GOLDEN, "engine_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def v8_dir():
    return os.path.join(GOLDEN, "v8SegmentPersistDir")


@pytest.fixture(scope="session")
def sample_dirs(tmp_path_factory):
    """TestIndex segment written with every codec/bitmap combination the engine reads."""
    import make_sample_segment
    out = {}
    base = tmp_path_factory.mktemp("sample")
    for bitmap in ("concise", "roaring"):
        for comp in ("lz4", "uncompressed", "none"):
            out[(bitmap, comp)] = make_sample_segment.build(str(base / f"{bitmap}_{comp}"), REPO, bitmap, comp)
    return out


@pytest.fixture(scope="session")
def basic_dirs(tmp_path_factory, DG):
    """Three small basic-schema segments per layout (synthetic, seeded)."""
    base = tmp_path_factory.mktemp("basic")
    out = {}
    for bitmap, comp in (("concise", "lz4"), ("roaring", "lz4"), ("concise", "uncompressed"), ("roaring", "none")):
        out[(bitmap, comp)] = DG.write_basic_dataset(str(base / f"{bitmap}_{comp}"), 3, 40_000, bitmap=bitmap,
                                                     compression=comp, lz4_mode="fast")
    return out
