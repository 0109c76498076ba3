"""Test-only CPU oracle for the PhotoHive_DSP hot path (see oracle/phd_oracle.h).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package; the product (photohive_dsp_amd) never does.
"""
