"""TEST INFRASTRUCTURE ONLY: CPU oracle + reference build (see oracle/oracle.py)."""
