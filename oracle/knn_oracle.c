/* placeholder, filled later */
