"""``har`` — MI355X-native human-activity-recognition framework.

The source tree lives in ``activity-recognition-using-apache-spark_amd/`` (a
directory name that is not a valid Python identifier).  This package points its
``__path__`` there, so ``import har.models.logreg`` resolves to
``activity-recognition-using-apache-spark_amd/models/logreg.py``.

Capability parity target: the single PySpark script ``Main/main.py`` of
Lohitanvita/Activity-Recognition-Using-Apache-Spark.
"""
import os as _os

_SRC = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                     "activity-recognition-using-apache-spark_amd")
__path__ = [_SRC]  # noqa: F821  (package path redirection)
__version__ = "0.1.0"

REPO_ROOT = _os.path.dirname(_SRC)
