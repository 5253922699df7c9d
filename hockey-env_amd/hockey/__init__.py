"""Drop-in alias: ``import hockey.hockey_env as h_env`` resolves to the MI355X implementation."""
