"""apps"""
