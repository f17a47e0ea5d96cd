"""Retrieval evaluation (Recall@k) over encoded page vectors."""
