"""Data-plane operators: HIP kernel wrappers (``nfdp``), packet crafting (``packets``)."""
