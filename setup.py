"""Package metadata + the native-build hook: ``build_py`` first builds the native libraries (ops/build.py: gfx950
HIP kernels + host C++, skipped when their build-id stamps are current) so the wheel carries stamped, up-to-date
libraries next to the sources the loaders check them against. Console scripts = the reference's five drivers
(GameTrainingDriver, GameScoringDriver, legacy Driver, FeatureIndexingDriver, NameAndTermFeatureBagsDriver) plus
the libsvm -> Avro converter."""
import os
import sys

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from photon_ml_amd.ops.build import build_all
        if os.environ.get("PML_SKIP_NATIVE_BUILD") != "1":
            build_all(verbose=True)
        super().run()


setup(
    name="photon-ml-amd",
    version="0.5.0",
    description="GLM and GAME (GLMix) training engine for AMD Instinct MI355X with Photon ML's drivers, "
                "estimator API and Avro formats",
    long_description=open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "README.md")).read(),
    long_description_content_type="text/markdown",
    python_requires=">=3.10",
    install_requires=["torch", "numpy", "scipy", "pyyaml", "pandas"],
    packages=find_packages(include=["photon_ml_amd", "photon_ml_amd.*"]),
    # the loaders check every library's build id against these sources (ops/build.py), so they ship together
    package_data={"photon_ml_amd": ["ops/_lib/*.so", "io/_lib/*.so", "ops/csrc/*.hip", "ops/csrc/*.h",
                                    "io/csrc/*.cpp"]},
    entry_points={"console_scripts": [
        "game-training = photon_ml_amd.cli.game_training:main",
        "game-scoring = photon_ml_amd.cli.game_scoring:main",
        "photon-ml = photon_ml_amd.cli.driver:main",
        "feature-indexing = photon_ml_amd.cli.feature_tools:indexing_main",
        "feature-bags = photon_ml_amd.cli.feature_tools:bags_main",
        "libsvm-to-avro = photon_ml_amd.tools.libsvm_to_avro:main",
    ]},
    cmdclass={"build_py": BuildNative},
)
