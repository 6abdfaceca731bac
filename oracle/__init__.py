"""CPU oracle (test infrastructure only; see oracle/raster_oracle.c)."""
