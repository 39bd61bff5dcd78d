import os
import sys

from . import _WORKER_ENV, _worker_main

if os.environ.get(_WORKER_ENV) == "1":
    _worker_main(sys.argv[1])
