"""Drop-in entry points with the reference's file names (program/research_questions/*.py).

Run from the directory that should receive ``data/result_data`` (the reference's CWD contract):
    FZ_DATA=<columnar or CSV-export dir> python -m tse_amd.research_questions.rq1_detection_rate
"""
