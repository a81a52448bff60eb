"""Test-only stand-in for compressai 1.2.6 (absent from this image, no network).

It restates the published semantics of the few compressai pieces the reference
imports, so that the reference's own Python (/root/reference/MLIC++) can run on
CPU in this container and produce golden fixtures (oracle/gen_golden.py).  It is
never shipped to the GPU box and never imported by the product.
"""
