"""TEST INFRASTRUCTURE ONLY: the CPU oracle package (see rt_oracle.c). Never imported by the product."""
