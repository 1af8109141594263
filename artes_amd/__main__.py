"""``python -m artes_amd <atmosphere> <photons> -o <output> [-k key=value]...`` (drop-in for ./bin/ARTES)."""

from .runner import main

raise SystemExit(main())
