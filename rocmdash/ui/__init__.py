"""Streamlit page (reference app.py:247-486)."""
