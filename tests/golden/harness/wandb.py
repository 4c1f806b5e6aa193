"""Placeholder so the reference's humanoid.algo package imports (wandb is unused on the env path)."""
