"""Packaging shim for setuptools < 61, which ignores pyproject.toml's
[project] table: the metadata and the ``numcodecs.codecs`` entry points are
read from pyproject.toml (the single source) and passed to setup().  Newer
setuptools reads [project] itself and this file only calls setup().
"""

import os

import setuptools
from setuptools import setup

_HERE = os.path.dirname(os.path.abspath(__file__))


def _legacy_kwargs():
    try:
        import tomllib
    except ImportError:  # Python 3.10
        import tomli as tomllib
    with open(os.path.join(_HERE, "pyproject.toml"), "rb") as f:
        cfg = tomllib.load(f)
    proj = cfg["project"]
    eps = {
        group: [f"{name} = {target}" for name, target in table.items()]
        for group, table in proj.get("entry-points", {}).items()
    }
    return dict(
        name=proj["name"],
        version=proj["version"],
        description=proj["description"],
        python_requires=proj["requires-python"],
        install_requires=proj.get("dependencies", []),
        packages=cfg["tool"]["setuptools"]["packages"],
        package_data=cfg["tool"]["setuptools"]["package-data"],
        entry_points=eps,
    )


if int(setuptools.__version__.split(".")[0]) < 61:
    setup(**_legacy_kwargs())
else:
    setup()
