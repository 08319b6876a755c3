"""Oracle package (test infrastructure only; see oracle.py / gs_oracle.c)."""
