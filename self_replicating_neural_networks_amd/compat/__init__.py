"""Drop-in modules named like the reference's (``network``, ``soup``, ``experiment``,
``util``).  ``enable()`` puts this directory on ``sys.path`` so reference-style scripts
(``from soup import *``) run unchanged on the MI355X engine."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def enable():
    if HERE not in sys.path:
        sys.path.insert(0, HERE)
